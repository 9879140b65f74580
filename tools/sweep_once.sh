for v in "engine.mtl.MTLProgram.SIDE_WGRAD_GRID=384" "engine.mtl.MTLProgram.SIDE_WGRAD_GRID=768" "engine.lowering.LoweredProgram.WGRAD_MAX_BATCHES_S0=2" "engine.core.ConvLayer.LEAN_BLOCKS=256" "engine.core.ConvLayer.LEAN_BLOCKS=1024"; do
  echo "=== $v"
  bash tools/gpu_session.sh ab "" "$v" 2 MTL || exit 1
  for f in gpurun_out/ab_MTL_A1.log gpurun_out/ab_MTL_B1.log gpurun_out/ab_MTL_A2.log gpurun_out/ab_MTL_B2.log; do grep -o '"value": [0-9.]*' $f; done | tr '\n' ' '; echo
done
