#!/bin/bash
# split map (parse kernel + signature-pass kernel): fused-map parity with the split (default) and the
# fused kernel, smoke, map A/B split vs fused (and vs lib_v1), then the headline bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd $R; O=gpurun_out/c6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -v -k "fused or golden or baseline_c1 or two_word or parse_line or full_size" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
FASTKMER_SPLIT_MAP=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t0.log 2>&1 || { tail -40 $O/t0.log; exit 1; }
tail -2 $O/t0.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
for r in 1 2; do
  for sp in 1 0; do
    FASTKMER_SPLIT_MAP=$sp FK_MAP_REPS=9 timeout -k 10 120 python -u scripts/map_once.py > $O/map_$sp.$r.txt 2>&1 || { tail $O/map_$sp.$r.txt; exit 1; }
    echo "split=$sp run $r: $(tail -1 $O/map_$sp.$r.txt)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/mp -o run -- python3 $R/scripts/map_once.py > $R/$O/mp.log 2>&1 || { tail -20 $R/$O/mp.log; exit 1; }
python3 $R/scripts/kstats.py $R/$O/mp/run_kernel_stats.csv 6
cd $R
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
cat $O/c1.json
