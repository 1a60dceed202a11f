#!/bin/bash
# Experimental build with several source files recompiled under extra flags, linked with the
# product objects of the other files into stratum-dsp_amd/lib_exp/lib_<name>.so:
#   bash tools/build_exp2.sh <name> "<file.hip>:<flags>" ["<file.hip>:<flags>" ...]
set -e
cd "$(dirname "$0")/../stratum-dsp_amd"
name=$1; shift
make -s -j8 >/dev/null
mkdir -p lib_exp build/exp
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-result -fno-slp-vectorize -I$(pwd)/csrc"
objs=""
skip=""
for spec in "$@"; do
  f=${spec%%:*}; fl=${spec#*:}
  base=$(basename $f .hip)
  extra=""
  /opt/rocm/bin/hipcc $HIPFLAGS $extra $fl -c csrc/$f -o build/exp/${base}_$name.o &
  objs="$objs build/exp/${base}_$name.o"
  skip="$skip build/$base.o"
done
wait
others=""
for o in build/*.o; do case " $skip " in *" $o "*) ;; *) others="$others $o";; esac; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib_exp/lib_$name.so $others $objs
echo lib_exp/lib_$name.so
