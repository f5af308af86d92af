"""The Python side of the gfx950 op wrappers (dmcp/ops/hip.py) run on the CPU
against a recording stand-in for the kernel library: every argument check,
workspace size and launch argument list of the GPU path executes here (a
wrapper's own bug -- an unbound name, a wrong argument count -- would
otherwise surface only on the GPU box).  The kernels themselves are checked
against fp32 by the ``gpu`` tests."""
import pytest
import torch


class _FakeLib:
    def __init__(self):
        self.calls = []

    def __getattr__(self, name):
        def fn(*args):
            self.calls.append((name, args))
            return 0
        return fn


@pytest.fixture
def dry(monkeypatch):
    from dmcp.ops import hip
    fake = _FakeLib()
    real_req = hip._req

    def req(t, dtype, name):  # the dtype / layout checks, without the device check
        if t.dtype != dtype:
            raise hip.HipOpsError(f"{name}: expected {dtype}, got {t.dtype}")
        if not t.is_contiguous():
            raise hip.HipOpsError(f"{name}: tensor must be contiguous")
    monkeypatch.setattr(hip, "_req", req)
    monkeypatch.setattr(hip, "_stream", lambda: None)
    monkeypatch.setattr(hip, "lib", lambda: fake)
    assert real_req is not req
    return hip, fake


def _bf(*shape):
    return torch.zeros(shape, dtype=torch.bfloat16)


@pytest.mark.parametrize("with_prefix", [False, True])
@pytest.mark.parametrize("with_fork", [False, True])
def test_decode_attention_launch_arguments(dry, with_prefix, with_fork):
    hip, fake = dry
    from dmcp.ops.reference import SharedPrefix
    B, Hq, Hkv, D, MAXS, S = 40, 32, 8, 64, 1024, 9
    q = _bf(B, Hq, D)
    kc, vc = _bf(S, Hkv, MAXS, D), _bf(S, Hkv, MAXS, D)
    slot = torch.zeros(B, dtype=torch.int32)
    lens = torch.ones(B, dtype=torch.int32)
    fork = torch.zeros(S, 2, dtype=torch.int32) if with_fork else None
    pre = SharedPrefix(kc[S - 1], vc[S - 1], torch.tensor([7], dtype=torch.int32)) if with_prefix else None
    out = hip.decode_attention(q, kc, vc, slot, lens, 0.125, prefix=pre, splits=3, fork=fork)
    name, args = fake.calls[-1]
    assert name == "dmcp_decode_attention" and len(args) == 25 and out.shape == q.shape
    ps = hip.prefix_mfma_splits(B, Hq // Hkv, Hkv) if with_prefix else 0
    assert args[20] == ps
    if with_prefix:  # a workspace without room for the prefix partials is refused, never overrun
        ws = hip.decode_workspace(B, Hq, Hkv, D, MAXS, "cpu", prefix_slots=0)
        with pytest.raises(hip.HipOpsError):
            hip.decode_attention(q, kc, vc, slot, lens, 0.125, workspace=ws, prefix=pre, splits=3, fork=fork)


def test_prefill_varlen_launch_arguments(dry):
    hip, fake = dry
    Hq, Hkv, D, MAXS, S = 32, 8, 64, 4096, 8
    offsets, slots, starts = [0, 100, 300], [1, 2], [1119, 1119]
    q = _bf(300, Hq, D)
    kc, vc = _bf(S, Hkv, MAXS, D), _bf(S, Hkv, MAXS, D)
    for _ in range(2):  # the second call reuses the work list built by the first
        hip.prefill_attention_varlen(q, kc, vc, offsets, slots, starts, 0, [1119, 1119], 0.125)
        name, args = fake.calls[-1]
        assert name == "dmcp_prefill_varlen" and len(args) == 17
    assert args[8] == sum(-(-T * 4 // hip.VARLEN_COLS) for T in (100, 200))


@pytest.mark.parametrize("M", [40, 320, 610])
def test_decode_gemm_wrappers_launch(dry, M):
    """The decode step's fused GEMM wrappers (weight-streaming up to 512 rows,
    large-tile above) with Llama-3.2-1B projection shapes."""
    hip, fake = dry
    H, I, Hq, Hkv, D, MAXS = 2048, 8192, 32, 8, 64, 1024
    Q = (Hq + 2 * Hkv) * D
    x = _bf(M, H)
    pos = torch.zeros(M, dtype=torch.int32)
    slot = torch.zeros(M, dtype=torch.int32)
    cs = torch.zeros(MAXS, D // 2, 2, dtype=torch.float32)
    kc, vc = torch.zeros(4, Hkv, MAXS, D, dtype=torch.uint8), torch.zeros(4, Hkv, MAXS, D, dtype=torch.uint8)
    resid, nw = _bf(M, H), _bf(H)
    V = 128256
    masks = torch.zeros(2, (V + 31) // 32, dtype=torch.int32)
    midx = torch.zeros(M, dtype=torch.int32)
    if M <= hip.WGEMM_MAX_ROWS:
        ws = hip.wgemm_workspace(M, Q, "cpu")
        hip.wgemm_rope_kv(x, _bf(Q, H), pos, slot, cs, kc, vc, Hq, ws)
        hip.wgemm_resid_norm(x, _bf(H, H), resid, nw, 1e-5, ws)
        hip.wgemm_resid_norm(_bf(M, I), _bf(H, I), resid, nw, 1e-5, ws)
        hip.wgemm_swiglu(x, _bf(2 * I, H))
        hip.lm_head_argmax(x, _bf(V, H), masks, midx, workspace=hip.lm_head_workspace(V, "cpu", M))
    if M > 256 or M <= hip.TGEMM_MAX_ROWS:
        tw = torch.empty(16 * M * Q, dtype=torch.float32)
        hip.tgemm_rope_kv(x, _bf(Q, H), pos, slot, cs, kc, vc, Hq, tw)
        hip.tgemm_resid_norm(x, _bf(H, H), resid, nw, 1e-5, tw)
        hip.tgemm_swiglu(x, _bf(2 * I, H))
        hip.tgemm_lm_head_argmax(x, _bf(V, H), masks, midx, workspace=torch.empty(2 * (V // 64) * M,
                                                                                   dtype=torch.float32))
    assert fake.calls and all(isinstance(n, str) for n, _ in fake.calls)
