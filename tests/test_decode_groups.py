"""Row groups of the per-row decode attention (CPU).

``dmcp.ops.decode_groups`` builds the table; the kernel
(``dmcp/ops/csrc/dmcp_kernels.hip``: ``row_group`` / ``group_geom`` /
``decode_attn_mfma_kernel``) decodes it defensively and deals every row's
keys over its group's work items.  ``_kernel_cover`` below is a line-by-line
Python model of that decoding and dealing; the tests check that, for the
host's tables and for arbitrary garbage ones, every key of every live row is
attended exactly once, from the cache bytes the row's fork-table view names
-- the property that makes grouping a pure performance choice (the GPU tests
compare the kernel's numbers against the fp32 reference).
"""
from __future__ import annotations

import numpy as np
import pytest

from dmcp.ops import hip

KMAX = 4


def _row_group(b, g7, g8, B, cap):
    if g7 is None:
        return [b], 0
    v = int(g7[b])
    lead = v & 0xFFFF
    if lead != b:
        if lead < B and (int(g7[lead]) & 0xFFFF) == lead:
            w = int(g8[lead]) & 0xFFFFFFFF
            ne = min(w & 3, cap - 1)
            if any(((w >> (2 + 10 * j)) & 1023) == b for j in range(ne)):
                return [], 0
        return [b], 0
    rows = [b]
    w = int(g8[b]) & 0xFFFFFFFF
    ne = min(w & 3, cap - 1)
    for j in range(ne):
        m = (w >> (2 + 10 * j)) & 1023
        if m < B and m != b and (int(g7[m]) & 0xFFFF) == b and m not in rows[1:]:
            rows.append(m)
    return rows, (v & 0xFFFFFFFF) >> 16


def _compat_end(P, pa, fa, sa, pb, fb, sb):
    lo, hi = max(P, min(fa, fb)), max(P, max(fa, fb))
    for k in (P, lo, hi):
        if (pa if k < fa else sa) != (pb if k < fb else sb):
            return k
    return 1 << 31


def _split_geom(Ls, splits, chunk):
    if Ls <= 0:
        return 0, 0
    n = min(splits, -(-Ls // chunk))
    part = (-(-Ls // n) + 31) & ~31
    return -(-Ls // part), part


def _geom(rows, nsplit, slot, seq_len, fork, prow, P0, max_seq, S, splits, chunk):
    d = []
    for b in rows:
        s = int(slot[b])
        L = min(int(seq_len[b]), max_seq) if 0 <= s < S else 0
        P = 0 if (prow is not None and not prow[b]) else P0
        ps, fe = s, 0
        if fork is not None and L > 0:
            p, e = int(fork[s, 0]), int(fork[s, 1])
            if e > 0 and 0 <= p < S and p != s:
                ps, fe = p, min(e, L)
        d.append((s, L, P, ps, fe))
    se = d[0][1]
    broken = d[0][1] <= 0
    for s, L, P, ps, fe in d[1:]:
        broken = broken or L <= 0 or P != d[0][2]
        se = min(se, L, _compat_end(d[0][2], d[0][3], d[0][4], d[0][0], ps, fe, s))
    se = d[0][2] if broken else max(se, d[0][2])
    Ls = se - d[0][2]
    nact, part = _split_geom(Ls, min(nsplit, splits), 32) if nsplit > 0 else _split_geom(Ls, splits, chunk)
    return d, se, broken, max(1, nact), part


def _kernel_cover(slot, seq_len, fork, prow, P0, max_seq, S, splits, chunk, groups, G):
    """{row: [(key, cache slot it is read from)]} as the kernel attends them,
    and the split count each row's output merges (one item per group and
    split; every key handed to one item)."""
    B = len(slot)
    cap = min(KMAX, 16 // G)
    g7, g8 = (None, None) if groups is None else (groups[0], groups[1])
    cover = {b: [] for b in range(B)}
    nact_of = {}
    for b in range(B):
        rows, nsplit = _row_group(b, g7, g8, B, cap)
        if not rows:
            continue
        d, se, broken, nact, part = _geom(rows, nsplit, slot, seq_len, fork, prow, P0, max_seq, S, splits, chunk)
        for r in rows:
            assert r not in nact_of, f"row {r} in two groups"
            nact_of[r] = nact
        P = d[0][2]
        s0, _, _, ps0, fe0 = d[0]
        for split in range(nact):
            if se > P:
                start = P + split * part
                end = min(se, start + part)
                for k in range(start, end):
                    src = ps0 if k < fe0 else s0
                    for r in rows:
                        cover[r].append((k, src))
            for j, r in enumerate(rows):
                if j % nact != split:
                    continue
                s, L, Pj, ps, fe = d[j]
                os_ = Pj if broken else se
                for k in range(os_, L):
                    cover[r].append((k, ps if k < fe else s))
    return cover, nact_of


def _truth(slot, seq_len, fork, prow, P0, max_seq, S):
    out = {}
    for b in range(len(slot)):
        s = int(slot[b])
        L = min(int(seq_len[b]), max_seq) if 0 <= s < S else 0
        P = 0 if (prow is not None and not prow[b]) else P0
        ps, fe = s, 0
        if fork is not None and L > 0:
            p, e = int(fork[s, 0]), int(fork[s, 1])
            if e > 0 and 0 <= p < S and p != s:
                ps, fe = p, min(e, L)
        out[b] = [(k, ps if k < fe else s) for k in range(P, L)] if L > 0 else []
    return out


def _scenario(rng, S=48, max_seq=600, P0=40):
    """Class heads (anchors) with method branches reading them in place,
    jump-forward rows of one slot, rows outside the prefix, padding."""
    fork = np.zeros((S, 2), dtype=np.int32)
    fork[:, 0] = np.arange(S)
    slots, lens, prow = [], [], []
    free = list(rng.permutation(S))
    while len(free) >= 6 and len(slots) < 90:
        anchor = int(free.pop())
        fe = int(rng.integers(P0 + 1, 300))
        inpre = int(rng.random() < 0.85)
        n_br = int(rng.integers(0, 6))
        members = [anchor]
        for _ in range(n_br):
            sl = int(free.pop())
            fork[sl] = (anchor, fe)
            members.append(sl)
        for sl in members:
            L = fe + int(rng.integers(1, 120)) if sl != anchor or n_br == 0 else fe + int(rng.integers(0, 120)) + 1
            for jump in range(int(rng.integers(1, 4))):  # jump rows: consecutive positions
                slots.append(sl)
                lens.append(min(max_seq, L + jump))
                prow.append(inpre)
    for _ in range(5):  # padding / bad slots
        slots.append(int(rng.choice([-1, S + 3])))
        lens.append(int(rng.integers(0, 50)))
        prow.append(1)
    perm = rng.permutation(len(slots))  # the engine's row order is arbitrary
    return (np.asarray(slots, np.int32)[perm], np.asarray(lens, np.int32)[perm], fork,
            np.asarray(prow, np.int32)[perm], P0, max_seq, S)


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("G", [4, 2, 8])
def test_host_groups_cover_every_key_once(seed, G):
    rng = np.random.default_rng(seed)
    slot, L, fork, prow, P0, max_seq, S = _scenario(rng)
    groups = hip.decode_groups(slot, L - 1, prow, fork, P0, 8 * G, 8, target_waves=int(rng.choice([256, 2048])))
    cover, nact = _kernel_cover(slot, L, fork, prow, P0, max_seq, S, 8, 256, groups, G)
    truth = _truth(slot, L, fork, prow, P0, max_seq, S)
    for b in range(len(slot)):
        assert sorted(cover[b]) == truth[b], f"row {b}"
    assert set(nact) == set(range(len(slot)))
    # the point of it: shared keys are read once per group
    single, _ = _kernel_cover(slot, L, fork, prow, P0, max_seq, S, 8, 256, None, G)
    reads = sum(len(v) for v in cover.values())
    assert reads == sum(len(v) for v in single.values())


def test_groups_share_the_class_head_keys():
    """An anchor + 3 branches + the anchor's jump row: one group of 4 rows
    (G = 4), the class head's keys [P, fork end) inside the shared range."""
    S, P0 = 8, 10
    fork = np.zeros((S, 2), dtype=np.int32)
    fork[:, 0] = np.arange(S)
    fork[[3, 4, 5]] = (2, 100)
    slot = np.array([2, 3, 4, 5, 2], np.int32)
    L = np.array([130, 120, 140, 101, 131], np.int32)
    prow = np.ones(5, np.int32)
    g = hip.decode_groups(slot, L - 1, prow, fork, P0, 32, 8, target_waves=64)
    cap_rows = {b for b in range(5) if (g[0, b] & 0xFFFF) == b}
    assert len(cap_rows) == 2  # 5 rows, at most 4 per group
    lead = [b for b in cap_rows if (g[1, b] & 3) == 3][0]
    rows, _ = _row_group(lead, g[0], g[1], 5, 4)
    d, se, broken, nact, part = _geom(rows, 1, slot, L, fork, prow, P0, 1024, S, 8, 256)
    assert not broken and se == 100 and len(rows) == 4


def test_garbage_tables_still_cover_every_row_once():
    rng = np.random.default_rng(7)
    slot, L, fork, prow, P0, max_seq, S = _scenario(rng)
    truth = _truth(slot, L, fork, prow, P0, max_seq, S)
    B = len(slot)
    for trial in range(200):
        g = np.empty((2, B), np.int32)
        if trial % 2:
            g[0] = rng.integers(0, B, B) | (rng.integers(0, 4, B) << 16)
        else:
            g[0] = rng.integers(-2**31, 2**31 - 1, B, dtype=np.int64).astype(np.int32)
        g[1] = rng.integers(-2**31, 2**31 - 1, B, dtype=np.int64).astype(np.int32)
        # some valid-looking member lists pointing back at their leaders
        for b in rng.integers(0, B, 6):
            ms = rng.integers(0, B, 3)
            g[0, b] = b
            g[1, b] = np.int64(3 | (ms[0] << 2) | (ms[1] << 12) | (ms[2] << 22)).astype(np.uint32).view(np.int32)
            for m in ms[:int(rng.integers(0, 4))]:
                g[0, m] = b
        cover, nact = _kernel_cover(slot, L, fork, prow, P0, max_seq, S, 8, 256, g, 4)
        for b in range(B):
            assert sorted(cover[b]) == truth[b], f"trial {trial} row {b}"


def test_group_split_counts_follow_the_keys():
    """Split counts: ~target_waves / Hkv items over the groups, in
    proportion to each group's keys, within [1, GROUP_MAX_SPLITS]."""
    S = 300
    fork = np.zeros((S, 2), np.int32)
    fork[:, 0] = np.arange(S)
    slot = np.arange(200, dtype=np.int32)
    L = np.where(np.arange(200) % 2 == 0, 2000, 200).astype(np.int32)
    g = hip.decode_groups(slot, L - 1, np.zeros(200, np.int32), fork, 0, 32, 8, target_waves=2048)
    ns = (g[0].astype(np.int64) & 0xFFFFFFFF) >> 16
    assert (ns >= 1).all() and (ns <= hip.GROUP_MAX_SPLITS).all()
    assert ns[::2].mean() > 2 * ns[1::2].mean()
    assert ((g[0] & 0xFFFF) == np.arange(200)).all()  # distinct slots, no fork: groups of one


def test_decode_groups_empty_and_cap():
    fork = np.zeros((4, 2), np.int32)
    fork[:, 0] = np.arange(4)
    assert hip.decode_groups(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32), fork, 0, 8, 8).shape \
        == (2, 0)
    # G = 16: one row per group
    g = hip.decode_groups(np.zeros(5, np.int32), np.arange(5, dtype=np.int32), np.ones(5, np.int32), fork, 0, 16, 1)
    assert ((g[0] & 0xFFFF) == np.arange(5)).all() and (g[1] == 0).all()
