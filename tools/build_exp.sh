#!/bin/bash
# Experimental builds of one source file (A/B and ablations), linked with the product objects
# into stratum-dsp_amd/lib_exp/lib_<name>.so (use with SDSP_LIB_PATH or tools/stft_probe.py):
#   bash tools/build_exp.sh <source.hip> <name> "<extra hipcc flags>" [<name> "<flags>" ...]
# <source.hip> is a file under csrc/ or any path to a variant of one (e.g. a `git show` of an
# older revision); the product object of the same basename is left out of the link.
set -e
cd "$(dirname "$0")/../stratum-dsp_amd"
src=$1; shift
base=$(basename $src .hip)
[ -f "$src" ] || src=csrc/$src
make -s -j8 >/dev/null
mkdir -p lib_exp build/exp
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-result -fno-slp-vectorize -I$(pwd)/csrc"
others=$(ls build/*.o | grep -v "build/$base.o")
names=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  names+=($name)
  /opt/rocm/bin/hipcc $HIPFLAGS $flags -c $src -o build/exp/${base}_$name.o &
done
wait
for name in "${names[@]}"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib_exp/lib_$name.so $others build/exp/${base}_$name.o
done
ls lib_exp
