#!/bin/bash
# complemented-norm pass (FK_MAPV 4): fused parity, smoke, map A/B vs FK_MAPV 3; count-stage PMC
# (every count kernel: VALU / LDS / HBM bytes) and kernel stats of one device-resident count.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=gpurun_out/c7; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -v -k "fused or golden or baseline_c1 or two_word or parse_line or random" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
bash scripts/ab_map.sh v3 || exit 1
bash scripts/pmc_count.sh r04 > $O/pmc_count.txt 2>&1 || { tail -20 $O/pmc_count.txt; exit 1; }
tail -80 $O/pmc_count.txt
cd /tmp && export TMPDIR=/tmp
FK_HT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/cnt -o run -- python3 $R/scripts/count_once.py > $R/$O/cnt.log 2>&1 || { tail -20 $R/$O/cnt.log; exit 1; }
python3 $R/scripts/kstats.py $R/$O/cnt/run_kernel_stats.csv 20
