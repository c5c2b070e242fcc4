"""Device placement of a context (include/fastkmer.h: all work of a context
runs on fk_config.device, whatever device the calling thread has current).

Every exported call that touches the GPU selects the context's device and
restores the caller's (fk_api.cpp DeviceGuard).  These tests use a context
from a thread other than the one that created it (the JNI shim's executor
threads do that) and, on a box with two GPUs, two contexts on different
devices driven alternately from one thread.
"""
import concurrent.futures as cf

import numpy as np
import pytest
import torch

import fastkmer_amd as fk
import oracle
from test_gpu_parity import assert_same_as_oracle

pytestmark = pytest.mark.gpu


def _fasta(seed):
    return fk.synth_fasta(3_000, 100, 200_000, seed=seed)


def test_context_used_from_another_thread():
    fasta = _fasta(21)
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    kc = fk.KmerCounter(28, 10, 3, 2048, False, 0, device=0)
    with cf.ThreadPoolExecutor(max_workers=2) as pool:
        pool.submit(kc.ingest, fasta).result()
        pool.submit(kc.finish).result()
        sizes = pool.submit(kc.bin_sizes).result()
    assert int(sizes.sum()) == int(ref.bin_sizes().sum())
    assert_same_as_oracle(kc, ref)
    # a second job on the same context from yet another thread
    with cf.ThreadPoolExecutor(max_workers=1) as pool:
        pool.submit(kc.ingest, fasta).result()
        pool.submit(kc.finish).result()
    assert_same_as_oracle(kc, ref)
    kc.close()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_two_devices_interleaved_in_one_thread():
    torch.cuda.set_device(1)
    fa, fb = _fasta(22), _fasta(23)
    ra, rb = oracle.OracleResult(fa, 28, 10, 2048), oracle.OracleResult(fb, 28, 10, 2048)
    ka = fk.KmerCounter(28, 10, 3, 2048, False, 0, device=0)
    kb = fk.KmerCounter(28, 10, 3, 2048, True, 0, device=1)
    ka.ingest(fa)
    kb.ingest(fb)
    ka.finish()
    kb.finish()
    assert torch.cuda.current_device() == 1  # the caller's device is restored after every call
    assert_same_as_oracle(ka, ra)
    assert_same_as_oracle(kb, rb, ordered=False)
    # and again with the jobs swapped between the contexts
    kb.ingest(fa)
    ka.ingest(fb)
    kb.finish()
    ka.finish()
    assert_same_as_oracle(kb, ra, ordered=False)
    assert_same_as_oracle(ka, rb)
    assert torch.cuda.current_device() == 1
    ka.close()
    kb.close()
    torch.cuda.set_device(0)


def test_device_input_then_host_input_on_one_context():
    # a context that mapped a borrowed device buffer (fk_ingest_device) takes host input for its
    # next job, and device input again after that (the JNI shim reuses one context per executor)
    fasta = _fasta(24)
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    buf = torch.frombuffer(bytearray(fasta), dtype=torch.uint8).to("cuda")
    torch.cuda.synchronize()
    with fk.KmerCounter(28, 10, 3, 2048, False, 0) as kc:
        kc.ingest_device(buf.data_ptr(), buf.numel())
        kc.finish()
        assert_same_as_oracle(kc, ref)
        kc.ingest(fasta)
        kc.finish()
        assert_same_as_oracle(kc, ref)
        kc.ingest_device(buf.data_ptr(), buf.numel())
        kc.finish()
        assert_same_as_oracle(kc, ref)


def test_bin_owners_with_grouped_emit():
    # fk_set_bin_owners with the grouped emit (the library's exchange layout): the (owner, local bin)
    # parts follow the new owners after a new fk_map, and the records per destination equal the
    # plain emit's under the same owners
    fasta = _fasta(25)
    owner = [(b + 1) % 2 for b in range(2048)]  # not the default bin % 2
    with fk.KmerCounter(28, 10, 3, 2048, False, 0, n_ranks=2, rank=0) as kc:
        kc.ingest(fasta)
        kc.map()
        plain = kc.set_bin_owners(owner)
    with fk.KmerCounter(28, 10, 3, 2048, False, 0, n_ranks=2, rank=0) as kc:
        kc.ingest(fasta)
        kc.set_grouped_emit(True)
        kc.set_bin_owners(owner)
        assert np.array_equal(kc.bin_owners(), owner)
        assert kc.map() == plain and sum(plain) > 0
