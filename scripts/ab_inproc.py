"""Interleaved A/B of FASTKMER_* env knobs in one process (min over repeats).
usage: python scripts/ab_inproc.py VAR=v1,v2,... [VAR2=...] [--reps 3] [--bytes N]"""
import os, sys, itertools
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import fastkmer_amd as fk
args = [a for a in sys.argv[1:] if "=" in a and not a.startswith("--")]
reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 3
nbytes = int(sys.argv[sys.argv.index("--bytes") + 1]) if "--bytes" in sys.argv else 1_000_000_000
B = int(sys.argv[sys.argv.index("--B") + 1]) if "--B" in sys.argv else 2048
K, M, RL = (55, 12, 150) if "--c4" in sys.argv else (28, 10, 100)
if "--c4" in sys.argv and "--B" not in sys.argv:
    B = 8192
axes = [(a.split("=")[0], a.split("=")[1].split(",")) for a in args]
combos = list(itertools.product(*[[(n, v) for v in vals] for n, vals in axes]))
best = {}
for rep in range(reps):
    for combo in combos:
        for n, v in combo:
            os.environ[n] = v
        kc = fk.KmerCounter(K, M, 3, B)
        kc.synth_device(nbytes // (RL + 14), RL, 100_000_000, seed=0x5EED)
        st = None
        for i in range(3):
            kc.finish()
            s = kc.stats()
            if st is None or s["ms_count"] < st["ms_count"]:
                st = s
        kc.close()
        key = " ".join(f"{n}={v}" for n, v in combo)
        prev = best.get(key)
        if prev is None or st["ms_count"] < prev["ms_count"]:
            best[key] = st
for key, st in best.items():
    print(f"k={K} B={B} {key}: count {st['ms_count']:.2f} ms  partition {st['ms_partition']:.2f}  sig {st['ms_signature']:.2f} "
          f"parse {st['ms_parse']:.2f}  distinct {st['distinct']}", flush=True)
