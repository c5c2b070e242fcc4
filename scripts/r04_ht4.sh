#!/bin/bash
# useHT k > 32: the 3072-slot mid tier between the 2048- and 6144-slot tables (FASTKMER_HT_HUGE).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=$R/gpurun_out/ht4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hash.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
probe() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u scripts/ht_probe.py > $O/probe_$n.txt 2>&1 || { tail -20 $O/probe_$n.txt; exit 1; }
  echo "== $n"; grep LDS $O/probe_$n.txt
}
probe base FK_X=0 || exit 1
probe h2600 FASTKMER_HT_HUGE=2600 || exit 1
probe h3500 FASTKMER_HT_HUGE=3500 || exit 1
probe b1500_h3000 FASTKMER_HT_BIG=1500 FASTKMER_HT_HUGE=3000 || exit 1
FK_BYTES=999999906 timeout -k 10 300 python -u scripts/ht_probe.py 28 10 2048 100 > $O/probe_c1.txt 2>&1 || { tail -20 $O/probe_c1.txt; exit 1; }
echo "== configs[1] useHT"; grep LDS $O/probe_c1.txt
