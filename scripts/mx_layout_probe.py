#!/usr/bin/env python3
"""Operand layout of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3) on the GPU box,
by one-hot probes through dmcp.ops.hip.mx_probe: for a one-hot A element
(lane, byte) and B holding coded values, which C entries light up and with
which B code; the same with A and B swapped; and which C entries each lane's
scale register scales.  Writes JSON for offline analysis."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main() -> int:
    from dmcp.ops import hip
    dev = "cuda"
    f8 = lambda v: torch.tensor(v, dtype=torch.float32).to(torch.float8_e4m3fn).view(torch.uint8)  # noqa: E731
    one = torch.full((64,), 127, dtype=torch.int32, device=dev)
    lanes = torch.arange(64)[:, None].expand(64, 32)
    bytes_ = torch.arange(32)[None, :].expand(64, 32)
    code1 = f8(((bytes_ % 16) + 1).float()).to(dev)            # byte % 16 + 1     (exact in e4m3)
    code2 = f8(((bytes_ // 16) + 2 * (lanes // 32) + 1).float()).to(dev)  # byte // 16, lane // 32
    out = {"a_onehot": [], "b_onehot": [], "scale_a": [], "scale_b": []}

    def nz(c):
        c = c.cpu()
        idx = (c != 0).nonzero().tolist()
        return [[l, r, float(c[l, r])] for l, r in idx]
    for la in range(64):
        for ja in range(32):
            a = torch.zeros(64, 32, dtype=torch.uint8, device=dev)
            a[la, ja] = int(f8(1.0))
            out["a_onehot"].append({"lane": la, "byte": ja, "c1": nz(hip.mx_probe(a, code1, one, one)),
                                    "c2": nz(hip.mx_probe(a, code2, one, one))})
            out["b_onehot"].append({"lane": la, "byte": ja, "c1": nz(hip.mx_probe(code1, a, one, one)),
                                    "c2": nz(hip.mx_probe(code2, a, one, one))})
    ones = torch.full((64, 32), int(f8(1.0)), dtype=torch.uint8, device=dev)
    for la in range(64):
        s = one.clone()
        s[la] = 128
        base = hip.mx_probe(ones, ones, one, one).cpu()
        out["scale_a"].append({"lane": la, "diff": nz(hip.mx_probe(ones, ones, s, one).cpu() - base)})
        out["scale_b"].append({"lane": la, "diff": nz(hip.mx_probe(ones, ones, one, s).cpu() - base)})
    # which data bytes a lane's scale multiplies: A one-hot at (lane la, byte j),
    # B all ones; the scale of lane ls doubled
    out["scale_member"] = []
    for la in (0, 32):
        for j in range(32):
            a = torch.zeros(64, 32, dtype=torch.uint8, device=dev)
            a[la, j] = int(f8(1.0))
            base = hip.mx_probe(a, ones, one, one).cpu().sum().item()
            hit = []
            for ls in range(64):
                s = one.clone()
                s[ls] = 128
                if hip.mx_probe(a, ones, s, one).cpu().sum().item() != base:
                    hit.append(ls)
            out["scale_member"].append({"lane": la, "byte": j, "scaled_by": hit})
    torch.cuda.synchronize()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/mx_layout.json", "w") as f:
        json.dump(out, f)
    print("ok", len(out["a_onehot"]))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
