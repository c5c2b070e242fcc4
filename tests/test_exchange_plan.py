"""Host arithmetic of the library's multi-rank exchange (fk_exchange_plan), no GPU.

Each exchange step every rank sends every other rank one message: its
records and k-mers per local bin of the receiver plus a flag word (bit 0: the
sender's last piece, bit 1: it retracts its earlier pieces).  The plan turns
the messages into the byte blocks of the step's all-to-all-v.  These tests
play whole jobs of several ranks through the plans: every block a rank
receives must be exactly the block its sender sends, blocks must tile the
buffers, and the closing rule (keep stepping until every rank has sent its
last piece) must end every rank on the same step whatever the piece counts.
"""
import numpy as np
import pytest

import fastkmer_amd as fk

FINAL, RETRACT = 1, 2


def messages(rng, world, parts, flags):
    """m[s, d] = rank s's message to rank d."""
    m = np.zeros((world, world, 2 * parts + 1), dtype=np.uint64)
    m[:, :, :parts] = rng.integers(0, 50, (world, world, parts))
    m[:, :, parts:2 * parts] = m[:, :, :parts] * rng.integers(1, 17, (world, world, parts))
    for s in range(world):
        m[s, :, 2 * parts] = flags[s]
    return m


@pytest.mark.parametrize("world,parts,rb", [(1, 3, 16), (2, 5, 16), (3, 4, 24), (8, 1024, 16)])
def test_plan_blocks_match_between_ranks(world, parts, rb):
    rng = np.random.default_rng(world * 100 + parts)
    m = messages(rng, world, parts, [0] * world)
    plans = [fk.exchange_plan(m[r], m[:, r], rb) for r in range(world)]
    for r, (so, sb, ro, rbytes, fin) in enumerate(plans):
        assert not fin
        # send blocks: destination-major, each = the records of the message times the record size
        assert np.array_equal(sb, m[r, :, :parts].sum(axis=1) * rb)
        assert np.array_equal(so, np.concatenate([[0], np.cumsum(sb)[:-1]]))
        assert np.array_equal(ro, np.concatenate([[0], np.cumsum(rbytes)[:-1]]))
        for s in range(world):
            assert rbytes[s] == plans[s][1][r], f"rank {r} expects {rbytes[s]} B from {s}"


def test_plan_final_and_retract_flags():
    world, parts = 3, 2
    rng = np.random.default_rng(3)
    m = messages(rng, world, parts, [FINAL, FINAL | RETRACT, 0])
    assert not fk.exchange_plan(m[0], m[:, 0], 16)[4]
    m = messages(rng, world, parts, [FINAL, FINAL | RETRACT, FINAL])
    assert all(fk.exchange_plan(m[r], m[:, r], 16)[4] for r in range(world))
    bad = messages(rng, world, parts, [RETRACT, 0, 0])  # a retract only comes with the last piece
    with pytest.raises(fk.FastKmerError):
        fk.exchange_plan(bad[1], bad[:, 1], 16)
    bad = messages(rng, world, parts, [8, 0, 0])
    with pytest.raises(fk.FastKmerError):
        fk.exchange_plan(bad[1], bad[:, 1], 16)


@pytest.mark.parametrize("pieces", [[3, 0, 5, 1], [0, 0], [7], [2, 2, 2, 2, 2, 2, 2, 9]])
def test_job_steps_close_together(pieces):
    """Ranks with different numbers of pieces: rank r sends pieces[r] pieces, then its
    last one (flag FINAL), then empty FINAL steps until the plan reports every rank
    final.  Every rank must stop on the same step and receive each sender's records once."""
    world, parts, rb = len(pieces), 6, 16
    rng = np.random.default_rng(sum(pieces) + world)
    sent_total = np.zeros((world, world), dtype=np.int64)  # records s -> d over the job
    recv_total = np.zeros((world, world), dtype=np.int64)
    step, done = 0, [False] * world
    while not all(done):
        flags, m = [], np.zeros((world, world, 2 * parts + 1), dtype=np.uint64)
        for s in range(world):
            if step < pieces[s]:
                flags.append(0)
            else:
                flags.append(FINAL)
            if step <= pieces[s]:  # pieces, then the last piece; closing steps carry nothing
                m[s, :, :parts] = rng.integers(0, 9, (world, parts))
            m[s, :, 2 * parts] = flags[s]
        for r in range(world):
            so, sb, ro, rbytes, fin = fk.exchange_plan(m[r], m[:, r], rb)
            sent_total[r] += (sb // rb).astype(np.int64)
            recv_total[:, r] += (rbytes // rb).astype(np.int64)
            done[r] = fin
        assert len(set(done)) == 1, f"ranks disagree on the last step at step {step}"
        step += 1
    assert step == max(pieces) + 1
    assert np.array_equal(sent_total, recv_total)
