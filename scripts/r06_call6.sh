#!/bin/bash
# Round 6, 6th GPU call: (a) phase probes of the 128-bit wave tier at the configs[3] load (FK_W128_STOP builds:
# 0 = key loads only, 1 = + fingerprint dedupe, 2 = + claimers' check; full and useHT from the product
# library), kernel time of k_bucket_count128_wave<2,...> from rocprofv3 --stats; (b) staged pieces: 5 / 6
# pieces per job (FK_STAGE_MAXP builds lib_p5 / lib_p6) at configs[1], the configs[2] and configs[3] loads;
# (c) where the piece work falls against the landing input (job_pieces.py) for the 5-piece c4 line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r06f; mkdir -p $O
cd $R
B="--steps 4 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off"
export TMPDIR=/tmp
probe() {  # name, extra bench args, then env assignments
  local name=$1 extra=$2; shift 2
  (cd /tmp && timeout -k 10 240 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run -- \
    python3 $R/bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off $extra \
    > $O/prof_$name.json 2> $O/prof_$name.err) || { echo "probe $name failed"; tail -5 $O/prof_$name.err; return 1; }
  python3 $R/scripts/kstats.py $O/prof_$name/run_kernel_stats.csv 40 > $O/kstats_$name.txt
  echo "$name: $(grep -E 'count128_wave<2' $O/kstats_$name.txt | head -1)"
}
probe full "" X=1 || exit 1
probe ht "--use-ht" X=1 || exit 1
for v in 0 1 2; do probe stop$v "" FASTKMER_LIB=$R/fastkmer_amd/lib_w128stop$v/libfastkmer.so || exit 1; done
line() {  # name workload, then env assignments
  local name=$1 wl=$2; shift 2
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl $B > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms'].items()})" $O/$name.json $name
}
P5=FASTKMER_LIB=$R/fastkmer_amd/lib_p5/libfastkmer.so
P6=FASTKMER_LIB=$R/fastkmer_amd/lib_p6/libfastkmer.so
for wl in c4 c3; do
  line ${wl}_base $wl X=1 || exit 1
  line ${wl}_p5a $wl $P5 FASTKMER_PIECE_CUTS=0.4,0.65,0.82,0.93 || exit 1
  line ${wl}_p5b $wl $P5 FASTKMER_PIECE_CUTS=0.45,0.7,0.85,0.95 || exit 1
  line ${wl}_p6a $wl $P6 FASTKMER_PIECE_CUTS=0.4,0.62,0.78,0.89,0.96 || exit 1
done
line c2_base c2 X=1 || exit 1
line c2_p5a c2 $P5 FASTKMER_PIECE_CUTS=0.4,0.65,0.82,0.93 || exit 1
line c2_p6a c2 $P6 FASTKMER_PIECE_CUTS=0.4,0.62,0.78,0.89,0.96 || exit 1
line c4_base2 c4 X=1 || exit 1
line c3_base2 c3 X=1 || exit 1
(cd /tmp && timeout -k 10 240 env FASTKMER_LIB=$R/fastkmer_amd/lib_p5/libfastkmer.so FASTKMER_PIECE_CUTS=0.4,0.65,0.82,0.93 \
  rocprofv3 --kernel-trace --output-format csv -d $O/trace_c4p5 -o run -- python3 $R/bench.py --workload c4 --steps 1 \
  --warmup 1 --no-cpu-baseline --no-device-leg --c3-leg off > $O/trace_c4p5.json 2> $O/trace_c4p5.err) || { echo "trace failed"; exit 1; }
python3 $R/scripts/job_pieces.py $O/trace_c4p5/run_kernel_trace.csv 0.5 > $O/c4p5_pieces.txt; tail -14 $O/c4p5_pieces.txt
