"""Host-side launch planning of the gfx950 kernels (pure Python, no GPU):
the weight-streaming GEMM's (K slices, M parts) and the decode step's
attention splits must respect what the kernels assume -- a mis-planned
launch is either a device fault or a second, mostly idle wave of blocks."""
import pytest

from dmcp.ops import hip

SHAPES = {"qkv": (3072, 2048, False), "o": (2048, 2048, False), "down": (2048, 8192, False),
          "gate_up": (16384, 2048, True), "qkv_3b": (5120, 3072, False), "down_3b": (3072, 8192, False),
          "gate_up_3b": (16384, 3072, True)}


@pytest.mark.parametrize("M", [1, 16, 17, 64, 78, 128, 200, 320, 383, 384, 448, 500, 512])
@pytest.mark.parametrize("shape", list(SHAPES))
def test_wgemm_plan_fits_the_kernel(M, shape):
    N, K, swiglu = SHAPES[shape]
    S, mparts = hip.wgemm_plan(M, N, K, swiglu=swiglu)
    assert S >= 1 and mparts >= 1 and (S & (S - 1)) == 0 and S <= 8
    assert K % (64 * S) == 0                                  # whole 64-deep chunks per slice
    rows = (-(-M // mparts) + 15) // 16 * 16
    assert rows <= 256                                        # <= 4 16-row tiles per wave
    assert mparts <= max(1, -(-M // 16))                      # no empty M parts
    if swiglu:
        assert S == 1                                         # SwiGLU writes its output directly
    tiles = (N // 2 if swiglu else N) // 64
    blocks = tiles * mparts * S
    if M >= 384:  # one block per CU: no mostly idle trailing wave
        waves = -(-blocks // 256)
        assert blocks / (256 * waves) >= 0.5, (blocks, waves)


def test_wgemm_plan_keeps_the_measured_small_m_plans():
    # tuned on the GPU at 320 rows (profiles/wgemm_r3.txt)
    assert hip.wgemm_plan(320, 3072, 2048) == (2, 2)
    assert hip.wgemm_plan(320, 2048, 8192) == (4, 2)
    assert hip.wgemm_plan(320, 16384, 2048, swiglu=True) == (1, 2)


@pytest.mark.parametrize("rows", [1, 16, 78, 320, 512, 768])
def test_prefix_splits_within_the_workspace(rows):
    sp = hip.prefix_mfma_splits(rows, 4, 8)
    assert 1 <= sp <= hip.PREFIX_MFMA_MAX_SPLITS


@pytest.mark.parametrize("inter", [128, 256, 1408, 5632, 8192, 8192 + 64, 100])
@pytest.mark.parametrize("hidden", [256, 2048, 2048 + 64])
def test_tgemm_model_and_op_predicates_agree(inter, hidden):
    """The model enables the large-tile path (tgemm_shapes_ok) exactly when
    every projection passes the op's own check (tgemm_supported), so no
    step -- nor the decode-graph capture at engine start -- raises inside
    tgemm_swiglu (advisor r5: intermediate = 128 x odd was enabled by one and
    refused by the other)."""
    from dmcp.models.llm import LMConfig, tgemm_shapes_ok
    c = LMConfig(hidden=hidden, intermediate=inter, n_heads=hidden // 64, n_kv_heads=max(1, hidden // 256),
                 head_dim=64)
    ops_ok = (hip.tgemm_supported(c.qkv_dim, c.hidden) and hip.tgemm_supported(c.hidden, c.hidden)
              and hip.tgemm_supported(2 * c.intermediate, c.hidden, swiglu=True)
              and hip.tgemm_supported(c.hidden, c.intermediate))
    model_ok = tgemm_shapes_ok(c)
    assert model_ok == (ops_ok and c.qkv_dim <= 8192 and c.hidden <= 8192)



def test_device_ops_share_one_signature():
    """Every op dispatched by device (dmcp.ops.DEVICE_OPS) has the same
    parameters in the kernel bindings and the fp32 references, so a call
    means the same on either device."""
    import inspect
    from dmcp import ops
    from dmcp.ops import reference
    for name in ops.DEVICE_OPS:
        k = list(inspect.signature(getattr(hip, name)).parameters)
        r = list(inspect.signature(getattr(reference, name)).parameters)
        assert k == r, name
        assert list(inspect.signature(getattr(ops, name)).parameters) == k, name


def _varlen_items_loop(offsets, slots, starts, plens, G):
    """The varlen work list as the per-item loop built it before round 6."""
    from dmcp.ops import hip
    seq, items = [], []
    for i in range(len(slots)):
        a, b, st, sl, P = offsets[i], offsets[i + 1], starts[i], slots[i], plens[i]
        T = b - a
        seq.append((a, T, st, sl, P))
        for ct in range(-(-T * G // hip.VARLEN_COLS)):
            last_tok = min(T, ((ct + 1) * hip.VARLEN_COLS + G - 1) // G)
            items.append((st + last_tok, i, ct))
    items.sort(key=lambda x: -x[0])
    return len(items), [v for _, i, ct in items for v in (i, ct)] + [v for r in seq for v in r]


@pytest.mark.parametrize("seed", range(6))
def test_varlen_work_list_matches_the_item_loop(seed):
    """The vectorised varlen work list (built once per prefill) is the
    per-item loop's, item for item; bad sequences are refused."""
    import random
    from dmcp.ops import hip
    rng = random.Random(seed)
    n = rng.randint(1, 60)
    lens = [rng.choice([1, 2, 31, 32, 33, 127, 128, 560, 2000]) for _ in range(n)]
    offsets = [0]
    for T in lens:
        offsets.append(offsets[-1] + T)
    slots = rng.sample(range(64), n)
    plens = [rng.choice([0, 1119]) for _ in range(n)]
    starts = [p + rng.randint(0, 50) if p else rng.randint(0, 50) for p in plens]
    G = rng.choice([1, 2, 4, 8])
    key = (tuple(offsets), tuple(slots), tuple(starts), 63, tuple(plens), G, 64, 4096, "cpu")
    n_items, meta = hip._varlen_meta(key, "cpu")
    exp_n, exp = _varlen_items_loop(offsets, slots, starts, plens, G)
    assert n_items == exp_n and meta.tolist() == exp
    with pytest.raises(hip.HipOpsError):  # a prefix that does not precede its start
        hip._varlen_meta((tuple(offsets), tuple(slots), tuple(0 for _ in starts), 63, tuple([5] * n), G, 64, 4096,
                          "cpu"), "cpu")
    with pytest.raises(hip.HipOpsError):  # past the slot's positions
        hip._varlen_meta((tuple(offsets), tuple(slots), tuple(starts), 63, tuple(plens), G, 64, 100, "cpu"), "cpu")
