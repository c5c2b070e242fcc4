#!/bin/bash
# Round 6, 11th GPU call: phases of the 64-bit wave tier at the configs[2] load (FK_W64_STOP builds: 0 = key
# loads only, 1 = + dedupe, 2 = + read-back of the distinct keys; full and useHT from the product library),
# k_bucket_count64_wave<2,...> per launch from rocprofv3 --stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06k; mkdir -p $O
cd $R
export TMPDIR=/tmp
probe() {  # name, extra bench args, then env assignments
  local name=$1 extra=$2; shift 2
  (cd /tmp && timeout -k 10 240 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- \
    python3 $R/bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off $extra \
    > $O/prof_$name.json 2> $O/prof_$name.err) || { echo "probe $name failed"; tail -5 $O/prof_$name.err; return 1; }
  python3 $R/scripts/kstats.py $O/prof_$name/run_kernel_stats.csv 40 > $O/kstats_$name.txt
  echo "$name: $(grep -E 'count64_wave<2' $O/kstats_$name.txt | head -1)"
}
probe full "" X=1 || exit 1
probe ht "--use-ht" X=1 || exit 1
for v in 0 1 2; do probe stop$v "" FASTKMER_LIB=$R/fastkmer_amd/lib_w64stop$v/libfastkmer.so || exit 1; done
