#!/bin/bash
# Host-only AddressSanitizer + UBSan run of the decode front-end (CPU, this container): builds the
# host_*.hip sources as C++ with a small driver (tools/micro/decode_fuzz_main.cpp) and decodes the
# damaged files that tests/test_decode_robustness.py's generator writes (truncations and byte
# corruptions of every supported container).  Any sanitizer report fails the run.
#   bash tools/asan_decode.sh [variants per format, default 400]
set -e
N=${1:-400}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$(mktemp -d)
for f in host_decode host_flac host_formats host_alac host_vorbis host_mkv; do
  g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -x c++ -c $R/stratum-dsp_amd/csrc/$f.hip -o $O/$f.o -I$R/stratum-dsp_amd/csrc
done
g++ -fsanitize=address,undefined $R/tools/micro/decode_fuzz_main.cpp $O/host_*.o -o $O/fuzz
mkdir -p $O/in
(cd $R/tests && python3 - "$O/in" "$N" <<'PY'
import os, sys
import numpy as np
sys.path.insert(0, ".")
import conftest  # noqa: F401
import test_decode_robustness as tr
out, n = sys.argv[1], int(sys.argv[2])
for fmt, data in sorted(tr.FILES.items()):
    rng = np.random.default_rng(hash(fmt) % (1 << 32) + 7)
    for trial in range(n):
        buf = bytearray(data)
        if trial % 4 == 0:
            buf = buf[:int(rng.integers(0, len(buf)))]
        else:
            for _ in range(int(rng.integers(1, 12))):
                buf[int(rng.integers(0, len(buf)))] = int(rng.integers(0, 256))
        open(os.path.join(out, f"{fmt}_{trial}"), "wb").write(bytes(buf))
PY
)
UBSAN_OPTIONS=halt_on_error=1 $O/fuzz $O/in/* 2>&1 | tee $O/log | tail -3
! grep -q "runtime error\|AddressSanitizer" $O/log
rm -rf $O
