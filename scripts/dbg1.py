import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.getcwd() + "/tests")
import numpy as np, fastkmer_amd as fk, oracle
fa = (b">r1\nACGTTGCATGCATGCAACGTTAGCCGATCGATCGGATCCATGCANNACGTTGCATGCATGCAACGTTAGCCGATCGAT\n"
      b">r2\nATCGATCGGCTAACGTTGCATGCATGCAACGTACGTTGCA\n>r3\n" + b"G" * 30 + b"\n")
for name, data in [("kat", fa), ("synth", fk.synth_fasta(200, 100, 5000, seed=1))]:
    kc = fk.KmerCounter(28, 10, 3, 2048); kc.ingest(data); kc.finish()
    ref = oracle.OracleResult(data, 28, 10, 2048)
    st = kc.stats()
    print(name, "gpu kmers", st["kmers"], "sk", st["superkmers"], "distinct", st["distinct"], "pos", st["positions"],
          "| ref kmers", ref.total_kmers, "distinct", ref.distinct)
    s = kc.bin_sizes().astype(np.int64); r = ref.bin_sizes()
    print(" nonzero gpu", np.nonzero(s)[0][:10], s[np.nonzero(s)[0][:10]], " ref", np.nonzero(r)[0][:10], r[np.nonzero(r)[0][:10]])
    for b in np.nonzero(r)[0][:3]:
        print("  ref", b, list(ref.bin_dict(b).items())[:3], " gpu", list(kc.bin_dict(b).items())[:3])
