"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/fastkmer.h declares, validates configurations like the
reference (and fails loudly when no GPU is present), and the host helpers
mirror TestConfiguration / LocalTestKmerCounter."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import fastkmer_amd as fk


@pytest.fixture(scope="module", autouse=True)
def built():
    from fastkmer_amd import build
    build.build()


def test_exports_every_header_symbol():
    names = fk.header_functions()
    assert len(names) >= 20
    L = ctypes.CDLL(fk.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.check_output(["nm", "-D", "--defined-only", fk.LIB_PATH]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(names) <= exported
    # nothing but the C-ABI leaks out of the shared object
    assert {n for n in exported if not n.startswith("fk_")} <= {"_init", "_fini"}


def test_abi_version():
    assert fk.lib().fk_abi_version() == 3 == fk.ABI_VERSION
    with open(fk.HEADER_PATH) as f:
        assert "#define FK_ABI_VERSION 3" in f.read()


def _header_struct_fields(name: str) -> list[tuple[str, str]]:
    import re
    with open(fk.HEADER_PATH) as f:
        text = f.read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), text, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    return re.findall(r"(int32_t|uint64_t|double)\s+(\w+);", body)


@pytest.mark.parametrize("name,cls", [("fk_config", fk.fk_config), ("fk_stats", fk.fk_stats)])
def test_ctypes_structs_mirror_the_header(name, cls):
    """The ctypes mirrors of fk_config / fk_stats have the header's fields, in order, with its
    types (a layout change bumps FK_ABI_VERSION, see the header's policy)."""
    ctype = {"int32_t": ctypes.c_int32, "uint64_t": ctypes.c_uint64, "double": ctypes.c_double}
    want = [(n, ctype[t]) for t, n in _header_struct_fields(name)]
    assert want and [(n, t) for n, t in cls._fields_] == want


def test_error_codes_mirror_the_header():
    import re
    with open(fk.HEADER_PATH) as f:
        codes = {int(v): n for n, v in re.findall(r"#define (FK_E_\w+) \((-\d+)\)", f.read())}
    assert codes == fk.ERRORS and codes[-7] == "FK_E_COMM"


@pytest.mark.parametrize("kw,ok", [
    (dict(k=28, m=10, x=3, B=2048), True),
    (dict(k=55, m=12, x=3, B=8192), True),
    (dict(k=64, m=15, x=1, B=1), True),
    (dict(k=28, m=10, x=0, B=2048), False),            # extractKXmers AIOOBE (SBKC:508)
    (dict(k=28, m=10, x=0, B=2048, use_ht=True), True),  # HT path never reads x
    (dict(k=28, m=16, x=3, B=2048), False),            # Int shift overflow (SBKC:50)
    (dict(k=65, m=10, x=3, B=2048), False),
    (dict(k=9, m=10, x=3, B=2048), False),
    (dict(k=28, m=10, x=3, B=0), False),
    (dict(k=28, m=10, x=3, B=2048, sequence_type=2), False),
    (dict(k=28, m=10, x=3, B=2048, n_ranks=2, rank=2), False),
    (dict(k=28, m=12, x=3, B=1 << 23), False),         # record header holds 22 bits of bin
])
def test_config_validation(kw, ok):
    if ok:
        fk.validate(**kw)
    else:
        with pytest.raises(fk.FastKmerError) as e:
            fk.validate(**kw)
        assert e.value.code == -1


def test_clamped_bins_and_output_dir():
    assert fk.clamped_bins(10, 2048) == 2048
    assert fk.clamped_bins(3, 2048) == 64
    assert fk.clamped_bins(15, 2**31 - 1) == 4**15
    c = fk.make_config(28, 10, 3, 2048)
    buf = ctypes.create_string_buffer(512)
    assert fk.lib().fk_output_dir(ctypes.byref(c), b"/out/", b"gallus", buf, 512) == 0
    tc = fk.TestConfiguration("in.fa", "/out/", 28, 10, 3, max_b=2048, prefix="gallus")
    assert buf.value.decode() == tc.outputDir == "/out/galluskk28_m10_x3_b2048_s0".replace("kk", "k")
    assert fk.TestConfiguration("a", "/o/", 21, 3, 2, max_b=2048).b == 64
    assert fk.TestConfiguration("a", "/o/", 21, 3, 2, debug=True).outputDir == "/tmp/k21_m3_x2_b64"


def test_record_bytes():
    assert fk.record_bytes_for_k(28) == 16
    assert fk.record_bytes_for_k(32) == 16
    assert fk.record_bytes_for_k(33) == 24
    assert fk.record_bytes_for_k(55) == 24


def test_synth_fasta_format_and_determinism():
    a = fk.synth_fasta(50, 100, 10_000, seed=7)
    b = fk.synth_fasta(50, 100, 10_000, seed=7)
    assert a == b and len(a) == 50 * 114
    recs = a.split(b"\n")
    assert recs[0] == b">r0000000000" and recs[2] == b">r0000000001"
    assert all(len(recs[i]) == 100 for i in range(1, 100, 2))
    assert set(b"".join(recs[1::2])) <= set(b"ACGTN")
    # a shard starting at read 20 is the tail of the full file
    assert fk.synth_fasta(30, 100, 10_000, seed=7, first_read=20) == a[20 * 114:]
    # error-free reads come from the virtual genome: every read is a substring
    # of it or of its reverse complement, so k-mers repeat across reads
    clean = fk.synth_fasta(400, 100, 2_000, seed=3, err_rate=0.0, n_rate=0.0)
    import collections
    reads = clean.split(b"\n")[1::2]
    kmers = collections.Counter(r[i:i + 21] for r in reads for i in range(80))
    assert max(kmers.values()) > 3


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(fk.FastKmerError) as e:
        fk.KmerCounter(28, 10)
    assert e.value.code == -3 and "no HIP device" in str(e.value)


def test_cli_usage_errors():
    fk_cli = fk.CLI_PATH
    r = subprocess.run([fk_cli], capture_output=True)
    assert r.returncode == 2 and b"usage" in r.stderr
    r = subprocess.run([fk_cli, "28", "16", "3", "2048", "0", "0", "in", "out", "p", "0", "0", "0"],
                       capture_output=True)
    assert r.returncode == 1 and b"invalid configuration" in r.stderr


def _lpt_reference(sizes, n):
    # MultiprocessorSchedulingPartitioner.solve (MultiprocessorSchedulingPartitioner.scala:35-69) on
    # the bins seen by the estimate, sorted by size descending (SBKC:1024); unseen bins hash to b % n
    # (getPartition, :17-24).  The reference's final shuffle of partition ids only relabels ranks.
    owner = [b % n for b in range(len(sizes))]
    loads = [0] * n
    for b in sorted((b for b in range(len(sizes)) if sizes[b]), key=lambda b: -sizes[b]):
        r = min(range(n), key=lambda q: loads[q])
        owner[b] = r
        loads[r] += sizes[b]
    return owner


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_lpt_owners_matches_reference_rule(n):
    import random
    rng = random.Random(n)
    sizes = [rng.choice([0, 0, rng.randint(1, 10), rng.randint(1, 100_000)]) for _ in range(500)]
    got = fk.lpt_owners(np.array(sizes, dtype=np.uint64), n)
    assert list(got) == _lpt_reference(sizes, n)
    loads = np.bincount(got, weights=sizes, minlength=n)
    assert loads.max() - loads.min() <= max(sizes)


def test_lpt_owners_validation():
    with pytest.raises(fk.FastKmerError):
        fk.lpt_owners(np.zeros(4, dtype=np.uint64), 0)


def test_jni_shim_matches_the_scala_natives_and_the_abi():
    """jni/fastkmer_jni.c defines one JNI function per @native method of
    skc.gpu.NativeKmerCounter and calls only symbols include/fastkmer.h declares
    (the shim is compiled only where a JDK exists; this image has none)."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    c_src = open(os.path.join(root, "jni", "fastkmer_jni.c")).read()
    scala = open(os.path.join(root, "jni", "skc", "gpu", "NativeKmerCounter.scala")).read()
    natives = set(re.findall(r"@native def (\w+)\(", scala))
    jni_funcs = set(re.findall(r"Java_skc_gpu_NativeKmerCounter_00024_(\w+)\(", c_src))
    assert natives and natives == jni_funcs
    declared = set(fk.header_functions())
    used = set(re.findall(r"\b(fk_\w+)\(", c_src))
    assert used and used <= declared, used - declared
