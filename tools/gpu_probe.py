"""One-shot MI355X probe: device info, hipcc .so loading into the torch process, MFMA lane maps,
and a reference-style eager PyTorch baseline of the Model A train step."""
import ctypes, os, sys, time, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.models import MTL_Net

print("device", torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).multi_processor_count, flush=True)
so = os.path.join(os.path.dirname(__file__), "mfma_probe.so")
lib = ctypes.CDLL(so)
A = torch.randint(-4, 5, (16, 32), device="cuda").float()
B = torch.randint(-4, 5, (32, 16), device="cuda").float()
C = torch.zeros(16, 16, device="cuda")
rc = lib.run_probe(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()),
                   ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
print("mfma rc", rc, "max err", (C - A @ B).abs().max().item(), flush=True)

def bench(model, bs, dtype, channels_last, steps=20, warm=5):
    model = model.cuda()
    if channels_last:
        model = model.to(memory_format=torch.channels_last)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5)
    x = torch.randn(bs, 1, 100, 250, device="cuda")
    if channels_last:
        x = x.to(memory_format=torch.channels_last)
    d = torch.randint(0, 16, (bs,), device="cuda"); e = torch.randint(0, 2, (bs,), device="cuda")
    crit = torch.nn.NLLLoss()
    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(dtype == "bf16")):
            o1, o2 = model(x)
            loss = crit(o1.float(), d) + crit(o2.float(), e)
        opt.zero_grad(); loss.backward(); opt.step()
    for _ in range(warm): step()
    torch.cuda.synchronize(); t = time.time()
    for _ in range(steps): step()
    torch.cuda.synchronize(); dt = (time.time() - t) / steps
    return dt
res = {}
for dtype in ["fp32", "bf16"]:
    for cl in [False, True]:
        torch.backends.cudnn.benchmark = True
        dt = bench(MTL_Net(), 32, dtype, cl)
        res[f"{dtype}_cl{int(cl)}"] = {"ms": dt * 1e3, "samples_per_s": 32 / dt}
        print(dtype, "channels_last" if cl else "nchw", f"{dt*1e3:.2f} ms/step  {32/dt:.0f} samples/s", flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/eager_baseline.json", "w"), indent=1)
