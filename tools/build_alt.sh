# Build the extension as of git revision REV into mtl_das_pytorch_amd/_ab/_mda_hip_REV.so (load it with
# MDA_EXT_PATH=... for A/B measurements against the working tree).   bash tools/build_alt.sh REV
set -e
rev=$1; d=$(mktemp -d); mkdir -p $d/pkg/csrc
for f in $(git ls-tree --name-only $rev mtl_das_pytorch_amd/csrc/); do git show $rev:$f > $d/pkg/csrc/$(basename $f); done
python $d/pkg/csrc/build.py --force > /dev/null
mkdir -p mtl_das_pytorch_amd/_ab
cp $d/pkg/_mda_hip*.so mtl_das_pytorch_amd/_ab/_mda_hip_$rev.so
rm -rf $d
echo mtl_das_pytorch_amd/_ab/_mda_hip_$rev.so
