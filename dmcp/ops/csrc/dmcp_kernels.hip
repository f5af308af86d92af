// dmcp HIP kernels for gfx950 (MI355X, CDNA4) -- the hot ops of the local
// enrichment model's decode/serve loop (dmcp/models/llm.py).
//
// Design rules followed (cdna_hip_programming.md): 64-lane waves, 256-thread
// blocks, every bf16 global access vectorized to 16 B (uint4) or 8 B (uint2)
// per lane (Guideline 13), fp32 accumulation, wave reductions with
// __shfl_xor over 64 lanes + one LDS hop across the 4 waves, RoPE from a
// host-precomputed cos/sin table (Appendix B), decode attention with K/V
// streamed straight to VGPRs (the 'GEMV / M <= 16' row: no LDS round trip),
// split-K over the sequence so B*Hkv*splits fills 256 CUs, and no
// allocation / synchronisation inside any launch function so every call can
// be captured into a hipGraph (Guideline 9).
//
// ABI: extern "C" launchers taking raw device pointers and a hipStream_t;
// they return hipError_t (0 = success).  Shapes are validated on the host
// side (dmcp/ops/hip.py) before any launch.
#include "dmcp_common.hpp"

// shared-prefix partials on the MFMA prefill kernel (prefill_attn.hip)
hipError_t dmcp_launch_prefix_partials(const uint16_t* q, const void* pk, const void* pv, const int32_t* plen,
                                       float* part_o, float* part_ml, int B, int Hkv, int G, int D, int ldk,
                                       int nsplit, int splits_total, float sl2, int kv8, hipStream_t st);

namespace {

// Per-row split geometry, shared by the per-row kernels and the combine:
// at most `splits` parts of >= `chunk` keys each, equal sizes rounded up to
// whole 32-key tiles (balanced work items instead of full chunks plus a
// short remainder).
struct SplitGeom {
    int nact, part;
};

__device__ __forceinline__ SplitGeom split_geom(int Ls, int splits, int chunk) {
    if (Ls <= 0) return {0, 0};
    int n = min(splits, (Ls + chunk - 1) / chunk);
    const int part = (((Ls + n - 1) / n) + 31) & ~31;
    n = (Ls + part - 1) / part;
    return {n, part};
}

// --------------------------------------------------------------------------
// 1. fused residual-add + RMSNorm:  h = x (+ residual);  residual <- h;
//    out = h * rsqrt(mean(h^2) + eps) * w.  One block per row, VPT 16-B
//    vectors per thread (H <= 256 * 8 * VPT).
// --------------------------------------------------------------------------
template <int VPT>
__global__ __launch_bounds__(kBlock) void add_rmsnorm_kernel(const uint16_t* __restrict__ x,
                                                            uint16_t* __restrict__ residual,
                                                            const uint16_t* __restrict__ w,
                                                            uint16_t* __restrict__ out, int H, float eps) {
    const int row = blockIdx.x;
    const int nvec = H >> 3;
    const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * H);
    uint4* rr = residual ? reinterpret_cast<uint4*>(residual + (size_t)row * H) : nullptr;
    const uint4* wr = reinterpret_cast<const uint4*>(w);
    // every global load (x, residual, weight) issued before the first use:
    // one memory round trip per launch instead of three (decode rows are few,
    // so the kernel is latency-, not bandwidth-bound)
    uint4 xv[VPT], rv[VPT], wv[VPT];
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            xv[i] = xr[idx];
            rv[i] = rr ? rr[idx] : make_uint4(0, 0, 0, 0);
            wv[i] = wr[idx];
        }
    }
    float h[VPT][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            unpack8(xv[i], h[i]);
            if (rr) {
                float r[8];
                unpack8(rv[i], r);
#pragma unroll
                for (int j = 0; j < 8; ++j) h[i][j] += r[j];
                uint4 packed = pack8(h[i]);
                rr[idx] = packed;
                unpack8(packed, h[i]);  // normalise the bf16-rounded stream (matches torch)
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += h[i][j] * h[i][j];
        }
    }
    __shared__ float red[kBlock / kWave];
    ss = wave_sum(ss);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < kBlock / kWave; ++k) tot += red[k];
    const float inv = rsqrtf(tot / (float)H + eps);
    uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * H);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            float wf[8], o[8];
            unpack8(wv[i], wf);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = h[i][j] * inv * wf[j];
            orow[idx] = pack8(o);
        }
    }
}

// --------------------------------------------------------------------------
// 2. RoPE (rotate-half) on q and k of a fused QKV row + KV-cache append.
//    qkv  [T, (Hq + 2 Hkv) * D]  ->  q_out [T, Hq, D]
//    k/v cache [S, Hkv, MAXS, D] written at (slot[t], :, pos[t], :)
//    cos_sin [max_pos, D/2] float2 (cos, sin)
//    KV8: the caches hold fp8 e4m3 (saturated), q stays bf16
// --------------------------------------------------------------------------
template <bool KV8>
__global__ __launch_bounds__(kBlock) void rope_kv_kernel(const uint16_t* __restrict__ qkv,
                                                        const int32_t* __restrict__ pos,
                                                        const int32_t* __restrict__ slot,
                                                        const float2* __restrict__ cos_sin,
                                                        uint16_t* __restrict__ q_out,
                                                        void* __restrict__ k_cache,
                                                        void* __restrict__ v_cache, int Hq, int Hkv,
                                                        int D, int max_seq, int max_pos, int num_slots) {
    const int t = blockIdx.x;
    const int p = pos[t];
    const int s = slot[t];
    const bool write_cache = (p >= 0 && p < max_seq && s >= 0 && s < num_slots);
    const int half = D >> 1;
    const int quads = half >> 2;  // groups of 4 rotary pairs
    const size_t row = (size_t)t * (size_t)(Hq + 2 * Hkv) * D;
    const float2* cs = cos_sin + (size_t)min(max(p, 0), max_pos - 1) * half;
    const int units = (Hq + Hkv) * quads;
    for (int u = threadIdx.x; u < units; u += kBlock) {
        const int hh = u / quads;
        const int d0 = (u - hh * quads) * 4;
        const uint16_t* src = qkv + row + (size_t)hh * D;
        float x1[4], x2[4], o1[4], o2[4];
        unpack4(*reinterpret_cast<const uint2*>(src + d0), x1);
        unpack4(*reinterpret_cast<const uint2*>(src + half + d0), x2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float2 c = cs[d0 + j];
            o1[j] = x1[j] * c.x - x2[j] * c.y;
            o2[j] = x2[j] * c.x + x1[j] * c.y;
        }
        if (hh < Hq) {
            uint16_t* dst = q_out + ((size_t)t * Hq + hh) * D;
            *reinterpret_cast<uint2*>(dst + d0) = pack4(o1);
            *reinterpret_cast<uint2*>(dst + half + d0) = pack4(o2);
            continue;
        }
        if (!write_cache) continue;
        const size_t kofs = (((size_t)s * Hkv + (hh - Hq)) * max_seq + p) * D;
        if constexpr (KV8) {
            uint8_t* dst = static_cast<uint8_t*>(k_cache) + kofs;
            *reinterpret_cast<uint32_t*>(dst + d0) = pack_fp8x4_bf16r(o1);
            *reinterpret_cast<uint32_t*>(dst + half + d0) = pack_fp8x4_bf16r(o2);
        } else {
            uint16_t* dst = static_cast<uint16_t*>(k_cache) + kofs;
            *reinterpret_cast<uint2*>(dst + d0) = pack4(o1);
            *reinterpret_cast<uint2*>(dst + half + d0) = pack4(o2);
        }
    }
    if (!write_cache) return;
    const int vvec = (Hkv * D) >> 3;
    const uint4* vsrc = reinterpret_cast<const uint4*>(qkv + row + (size_t)(Hq + Hkv) * D);
    for (int u = threadIdx.x; u < vvec; u += kBlock) {
        const int e = u << 3;
        const int kh = e / D;
        const int d = e - kh * D;
        const size_t vofs = (((size_t)s * Hkv + kh) * max_seq + p) * D + d;
        if constexpr (KV8)
            *reinterpret_cast<uint2*>(static_cast<uint8_t*>(v_cache) + vofs) = bf16x8_to_fp8x8(vsrc[u]);
        else
            *reinterpret_cast<uint4*>(static_cast<uint16_t*>(v_cache) + vofs) = vsrc[u];
    }
}

// --------------------------------------------------------------------------
// 3. decode attention (one query token per row), GQA, split-K: the per-row
//    MFMA kernel (3c below) writes fp32 partials (or the output directly
//    when a row fits one split and there is no shared prefix); the shared
//    prefix's partials come from the MFMA prefill kernel in prefix mode
//    (prefill_attn.hip); this kernel merges them.
// --------------------------------------------------------------------------
// Split-K merge.  One wave per (row, q head): lane = (4-output group
// dg = lane % (D/4), partial group pg = lane / (D/4)); each lane merges
// every (64/(D/4))-th partial with float4 loads issued 8 at a time, then
// the partial groups are merged across lanes with two shuffles.  A row's
// ~20 partials (shared-prefix splits + suffix splits) cost one memory
// round trip, on 4x more waves than a thread-per-output merge (which was
// latency-bound at 8-12 us per layer -- profiles/decode_step_r2_*).
// Rows whose own keys fit one split (nact <= 1) were finished by the main
// kernel (with a shared prefix it merges the prefix partials itself), so the
// pass runs only for steps of more than one split per row.  (A fused "last block merges" variant needs agent-scope release
// fences; on gfx950 each one writes back the XCD's L2 and made the kernel
// ~10x slower -- profiles/ROUND1_NOTES.md.)
template <int D>
__global__ __launch_bounds__(kBlock) void decode_attn_combine_kernel(const float* __restrict__ part_o,
                                                                    const float* __restrict__ part_ml,
                                                                    const int32_t* __restrict__ slot,
                                                                    const int32_t* __restrict__ seq_len,
                                                                    uint16_t* __restrict__ out, int B, int Hq,
                                                                    int max_seq, int chunk, int splits,
                                                                    int num_slots, const int32_t* __restrict__ plen,
                                                                    int ps_max, const int32_t* __restrict__ prow) {
    constexpr int U = 8;
    constexpr int DQ = D / 4;       // lanes per partial group
    constexpr int PG = kWave / DQ;  // partial groups per wave
    const int lane = threadIdx.x & (kWave - 1);
    const int dg = lane % DQ, pg = lane / DQ;
    const int P0 = plen ? max(0, *plen) : 0;
    const int splits_total = ps_max + splits;
    const int nwaves = gridDim.x * (kBlock / kWave);
    for (int w = blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave; w < B * Hq; w += nwaves) {
        const int b = w / Hq, qh = w - b * Hq;
        const int s = slot[b];
        const int L = (s >= 0 && s < num_slots) ? min(seq_len[b], max_seq) : 0;
        if (L <= 0) continue;  // padding row: zeroed by the main kernel
        // prow[b] == 0: a row outside the shared prefix (another project's
        // sequence) -- all its keys are its own; its prefix partials unused
        const int P = (prow && !prow[b]) ? 0 : P0;
        // the shared prefix's ps_max partials (prefill kernel in prefix mode;
        // splits past the prefix's end are empty and weigh 0)
        const int npre = P > 0 ? ps_max : 0;
        const int nact = split_geom(L - P, splits, chunk).nact;
        if (nact <= 1) continue;  // finished by the main kernel (directly, or merging the prefix partials)
        const int n = npre + nact;
        const size_t base = ((size_t)b * Hq + qh) * splits_total;
        float m = -1e30f, lt = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        for (int i0 = pg; i0 < n; i0 += U * PG) {
            float2 ml[U];
            float4 o4[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int i = i0 + j * PG;
                const size_t idx = base + (i < npre ? i : ps_max + (i - npre));
                if (i < n) {
                    ml[j] = *reinterpret_cast<const float2*>(part_ml + idx * 2);
                    o4[j] = *reinterpret_cast<const float4*>(part_o + idx * D + 4 * dg);
                } else {
                    ml[j] = make_float2(-1e30f, 0.f);
                    o4[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
            float mn = m;
#pragma unroll
            for (int j = 0; j < U; ++j) mn = fmaxf(mn, ml[j].x);
            const float ca = exp2f(m - mn);
            lt *= ca; a0 *= ca; a1 *= ca; a2 *= ca; a3 *= ca;
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const float cb = exp2f(ml[j].x - mn);
                lt += ml[j].y * cb;
                a0 += o4[j].x * cb; a1 += o4[j].y * cb; a2 += o4[j].z * cb; a3 += o4[j].w * cb;
            }
            m = mn;
        }
        // merge the PG partial groups (lanes dg, dg + DQ, ...)
#pragma unroll
        for (int msk = DQ; msk < kWave; msk <<= 1) {
            const float mo = __shfl_xor(m, msk, kWave);
            const float mn = fmaxf(m, mo);
            const float ca = exp2f(m - mn), cb = exp2f(mo - mn);
            lt = lt * ca + __shfl_xor(lt, msk, kWave) * cb;
            a0 = a0 * ca + __shfl_xor(a0, msk, kWave) * cb;
            a1 = a1 * ca + __shfl_xor(a1, msk, kWave) * cb;
            a2 = a2 * ca + __shfl_xor(a2, msk, kWave) * cb;
            a3 = a3 * ca + __shfl_xor(a3, msk, kWave) * cb;
            m = mn;
        }
        if (pg == 0) {
            const float inv = lt > 0.f ? 1.f / lt : 0.f;
            const float f[4] = {a0 * inv, a1 * inv, a2 * inv, a3 * inv};
            *reinterpret_cast<uint2*>(out + ((size_t)b * Hq + qh) * D + 4 * dg) = pack4(f);
        }
    }
}

// --------------------------------------------------------------------------
// 4. SwiGLU activation: out[t, i] = silu(gu[t, i]) * gu[t, I + i]
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void silu_mul_kernel(const uint16_t* __restrict__ gu,
                                                         uint16_t* __restrict__ out, int T, int I) {
    const int vpr = I >> 3;
    const size_t total = (size_t)T * vpr;
    for (size_t u = (size_t)blockIdx.x * kBlock + threadIdx.x; u < total; u += (size_t)gridDim.x * kBlock) {
        const size_t t = u / vpr;
        const int c = (int)(u - t * vpr) << 3;
        const uint16_t* row = gu + t * (size_t)(2 * I);
        float g[8], up[8], o[8];
        unpack8(*reinterpret_cast<const uint4*>(row + c), g);
        unpack8(*reinterpret_cast<const uint4*>(row + I + c), up);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = g[j] / (1.f + __expf(-g[j])) * up[j];
        *reinterpret_cast<uint4*>(out + t * (size_t)I + c) = pack8(o);
    }
}

// --------------------------------------------------------------------------
// 5. masked greedy sampling: ids[b] = argmax_{v allowed} logits[b, v]
//    mask: uint32 bit-sets of allowed tokens, ceil(V/32) words per row
//    (nullptr = all).  With mask_idx, row b uses mask row mask_idx[b]
//    (clamped to [0, n_masks)) of a small shared table -- the decode graph
//    selects the grammar state per row without an index_select; without it,
//    mask row b.  Ties resolve to the smallest index.
// --------------------------------------------------------------------------
__device__ __forceinline__ void argmax_take(float x, int v, float& best, int& bi) {
    if (x > best || (x == best && v < bi)) { best = x; bi = v; }
}

// One 1,024-thread block per row.  Whole 8-id chunks are read as one 16-B
// load each with the chunk's 8 mask bits (one byte of a mask word), MA_U
// chunks per thread issued before any is compared (indices clamped, the
// duplicates masked out), and each of a chunk's 8 positions keeps its own
// running (max, id): eight independent compare/select chains, no branch.
// Within one chain ids only grow, so a strict > keeps the lowest id of a
// tie; the chains and the threads merge with the explicit tie rule.  The
// element-wise loop this replaces (256 threads, one chain, a branch per id)
// took ~290 us per prefill batch at 128,256 ids
// (profiles/llama_engine_kernel_stats_r6.csv), ~42 us per row-block even
// with its loads vectorised: it was bound by its dependent compare chain,
// not by memory.  A row that is not 16-B aligned (ld % 8 != 0) and the ids
// past the last whole chunk take the element-wise loop.
constexpr int MA_T = 1024, MA_U = 2;

__global__ __launch_bounds__(MA_T) void masked_argmax_kernel(const uint16_t* __restrict__ logits,
                                                            const uint32_t* __restrict__ mask,
                                                            const int32_t* __restrict__ mask_idx, int n_masks,
                                                            int32_t* __restrict__ ids, int V, int ld, int nch) {
    const int b = blockIdx.x;
    const uint16_t* row = logits + (size_t)b * ld;
    int mr = b;
    if (mask_idx) {
        mr = mask_idx[b];
        mr = mr < 0 ? 0 : (mr >= n_masks ? n_masks - 1 : mr);
    }
    const uint32_t* mrow = mask ? mask + (size_t)mr * ((V + 31) >> 5) : nullptr;
    float bv[8];
    int bc[8];  // chunk index of bv[j] (id = 8 * chunk + j)
#pragma unroll
    for (int j = 0; j < 8; ++j) { bv[j] = -INFINITY; bc[j] = 0x0fffffff; }
    for (int c0 = threadIdx.x; c0 < nch; c0 += MA_T * MA_U) {
        uint4 q[MA_U];
        uint32_t mb[MA_U];
#pragma unroll
        for (int u = 0; u < MA_U; ++u) {
            const int c = min(c0 + u * MA_T, nch - 1);
            q[u] = *reinterpret_cast<const uint4*>(row + (size_t)c * 8);
            mb[u] = mrow ? (mrow[c >> 2] >> ((c & 3) * 8)) & 0xFFu : 0xFFu;
        }
#pragma unroll
        for (int u = 0; u < MA_U; ++u) {
            const int c = c0 + u * MA_T;
            const uint32_t m = c < nch ? mb[u] : 0u;
            const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float x = __uint_as_float((j & 1) ? (w[j >> 1] & 0xFFFF0000u) : (w[j >> 1] << 16));
                x = ((m >> j) & 1u) ? x : -INFINITY;
                const bool t = x > bv[j];
                bv[j] = t ? x : bv[j];
                bc[j] = t ? c : bc[j];
            }
        }
    }
    float best = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (bc[j] != 0x0fffffff) argmax_take(bv[j], bc[j] * 8 + j, best, bi);
    for (int v = nch * 8 + threadIdx.x; v < V; v += MA_T) {
        if (mrow && !((mrow[v >> 5] >> (v & 31)) & 1u)) continue;
        argmax_take(bf2f(row[v]), v, best, bi);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const float ob = __shfl_xor(best, m, kWave);
        const int oi = __shfl_xor(bi, m, kWave);
        argmax_take(ob, oi, best, bi);
    }
    __shared__ float sb[MA_T / kWave];
    __shared__ int si[MA_T / kWave];
    if ((threadIdx.x & (kWave - 1)) == 0) { sb[threadIdx.x / kWave] = best; si[threadIdx.x / kWave] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float B = sb[0];
        int I = si[0];
        for (int k = 1; k < MA_T / kWave; ++k) argmax_take(sb[k], si[k], B, I);
        ids[b] = (I == 0x7fffffff) ? 0 : I;
    }
}

// --------------------------------------------------------------------------
// 6. embedding gather: out[t, :] = table[clamp(ids[t]), :]
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void embedding_kernel(const uint16_t* __restrict__ table,
                                                          const int32_t* __restrict__ ids,
                                                          uint16_t* __restrict__ out, int T, int H, int V) {
    const int vpr = H >> 3;
    const size_t total = (size_t)T * vpr;
    for (size_t u = (size_t)blockIdx.x * kBlock + threadIdx.x; u < total; u += (size_t)gridDim.x * kBlock) {
        const size_t t = u / vpr;
        const int c = (int)(u - t * vpr);
        int id = ids[t];
        id = id < 0 ? 0 : (id >= V ? V - 1 : id);
        reinterpret_cast<uint4*>(out + t * (size_t)H)[c] = reinterpret_cast<const uint4*>(table + (size_t)id * H)[c];
    }
}

// --------------------------------------------------------------------------
// 7. decode-step inputs in one launch (one block per row): the row's token
//    (tok = src[r] >= 0 ? last_ids[src[r]] : tokens[r] -- the previous step's
//    selection still on the device, the engine's one-step pipeline), its
//    embedding row into the residual stream, the first RMSNorm of it into h
//    (skipped when h is null) and seq_len[r] = pos[r] + 1.  Replaces an
//    index_select / where / clamp / compare / embedding / clone / add_rmsnorm
//    / add chain of 7 launches per decode step.
// --------------------------------------------------------------------------
template <int VPT>
__global__ __launch_bounds__(kBlock) void decode_embed_norm_kernel(
    const uint16_t* __restrict__ table, const int32_t* __restrict__ tokens, const int32_t* __restrict__ src,
    const int32_t* __restrict__ last_ids, const int32_t* __restrict__ pos, const uint16_t* __restrict__ w,
    uint16_t* __restrict__ resid, uint16_t* __restrict__ h, int32_t* __restrict__ seq_len, int H, int V,
    int n_last, float eps, int32_t* __restrict__ mask_idx, const int32_t* __restrict__ mask_alt, int alt_token) {
    const int row = blockIdx.x;
    int id = tokens[row];
    if (src) {
        const int s = src[row];
        if (s >= 0) {
            id = last_ids[s < n_last ? s : n_last - 1];
            // grammar: a gathered token that closes a free string (the
            // engine's lone quote) switches this row's selection mask to the
            // next segment's -- the host learns the token only a step later
            if (mask_alt && threadIdx.x == 0 && id == alt_token) {
                const int a = mask_alt[row];
                if (a >= 0) mask_idx[row] = a;
            }
        }
    }
    id = id < 0 ? 0 : (id >= V ? V - 1 : id);
    if (threadIdx.x == 0) seq_len[row] = pos[row] + 1;
    const int nvec = H >> 3;
    const uint4* er = reinterpret_cast<const uint4*>(table + (size_t)id * H);
    uint4* rr = reinterpret_cast<uint4*>(resid + (size_t)row * H);
    uint4 xv[VPT], wv[VPT];
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            xv[i] = er[idx];
            if (h) wv[i] = reinterpret_cast<const uint4*>(w)[idx];
        }
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) rr[idx] = xv[i];
    }
    if (!h) return;
    float x[VPT][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            unpack8(xv[i], x[i]);
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += x[i][j] * x[i][j];
        }
    }
    __shared__ float red[kBlock / kWave];
    ss = wave_sum(ss);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < kBlock / kWave; ++k) tot += red[k];
    const float inv = rsqrtf(tot / (float)H + eps);
    uint4* orow = reinterpret_cast<uint4*>(h + (size_t)row * H);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            float wf[8], o[8];
            unpack8(wv[i], wf);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = x[i][j] * inv * wf[j];
            orow[idx] = pack8(o);
        }
    }
}

// One 32-key tile of a (slot, kv head): K rows as the S^T A operand (key
// kt + 16h + (lane&15), dims 32ks + 8*(lane>>4)) and the V tile (32 x D,
// contiguous) as 16-B chunks, chunk lane + 64r.  A full tile is addressed
// from one per-tile base plus compile-time offsets (no per-load 64-bit
// address math); the partial last tile of a split clamps every key to
// end-1 (in-bounds, finite; masked later).
template <int D, bool KV8>
struct KVTile;

template <int D>
struct KVTile<D, false> {
    uint4 k[2][D / 32];  // 8 bf16 per (half, k-step)
    uint4 v[D / 16];     // 8 bf16 per chunk
};

template <int D>
struct KVTile<D, true> {
    uint2 k[2][D / 32];  // 8 e4m3 per (half, k-step)
    uint4 v[D / 32];     // 16 e4m3 per chunk
};

// element offset -> byte address of a bf16 or fp8 cache
template <bool KV8>
__device__ __forceinline__ const char* kv_at(const void* base, size_t off) {
    return static_cast<const char*>(base) + off * (KV8 ? 1 : 2);
}

// A row's K/V bases: its own slot's, and -- a method branch -- its class
// head's slot (the parent), which holds the keys [.., fend) the branch
// shares: keys below fend are read there in place, never copied.
struct KVSrc {
    const void* k;
    const void* v;
    const void* pk;
    const void* pv;
    int fend;  // 0: no parent
};

template <int D, bool KV8>
__device__ __forceinline__ void load_kv_tile(const KVSrc& src, int kt, int end, int lane, KVTile<D, KV8>& t) {
    using KRaw = std::conditional_t<KV8, uint2, uint4>;
    constexpr int VE = KV8 ? 16 : 8;  // elements per V chunk
    constexpr int CPK = D / VE;       // V chunks per key
    constexpr int NV = 32 * D / VE / kWave;
    const bool par = kt + 32 <= src.fend;                // the whole tile is the parent's
    const bool mixed = !par && kt < src.fend;            // the tile straddles the fork point
    const void* kb = par ? src.pk : src.k;
    const void* vb = par ? src.pv : src.v;
    if (kt + 32 <= end && !mixed) {
        const char* kp = kv_at<KV8>(kb, (size_t)(kt + (lane & 15)) * D + 8 * (lane >> 4));
        const char* vp = kv_at<KV8>(vb, (size_t)kt * D + lane * VE);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int ks = 0; ks < D / 32; ++ks)
                t.k[h][ks] = *reinterpret_cast<const KRaw*>(kp + (16 * h * D + 32 * ks) * (KV8 ? 1 : 2));
#pragma unroll
        for (int r = 0; r < NV; ++r) t.v[r] = *reinterpret_cast<const uint4*>(vp + 16 * kWave * r);
        return;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int key = min(kt + 16 * h + (lane & 15), end - 1);
        const void* kk = key < src.fend ? src.pk : src.k;
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks)
            t.k[h][ks] = *reinterpret_cast<const KRaw*>(kv_at<KV8>(kk, (size_t)key * D + 32 * ks + 8 * (lane >> 4)));
    }
#pragma unroll
    for (int r = 0; r < NV; ++r) {
        const int ch = lane + kWave * r;
        const int key = min(kt + ch / CPK, end - 1);
        const void* vv = key < src.fend ? src.pv : src.v;
        t.v[r] = *reinterpret_cast<const uint4*>(kv_at<KV8>(vv, (size_t)key * D + (ch % CPK) * VE));
    }
}

// V tile layout in LDS: 32 key rows of D bf16, unpadded, with the 4-element
// quads of row r stored at quad index q ^ vswz(r).  The XOR leaves every
// 16-B store whole and makes both access patterns conflict-free
// (MI355X_MICROARCH.md §LDS bank rules):
//  * ds_read_b64_tr_b16 (2 x 32 lanes, bank (a/4) mod 64): a half reads 8
//    rows x one 4-quad d block; rows of equal parity share a bank window and
//    get distinct quad groups (bits 2-3 of the XOR, (r>>1)&3);
//  * ds_write_b128 of fp8-converted V (8 x 8 lanes, bank (a/4) mod 32): a
//    group stores rows r, r+1 at the same quads; bit 1 of the XOR (r&1) puts
//    the odd row in the other 16-B half of each 32-B window.
// The padded layout this replaces (144-B rows) measured ~1 conflict cycle per
// LDS instruction (profiles/pmc_decode_step_320rows_fp8_r3.txt).
// D=128 (a row is a whole 256-B bank row): quad groups XORed with r & 7 for
// the reads, and within a group the two 16-B halves swapped when the
// physical group has bit 2 set (vquad) -- an 8-lane fp8 store group is one
// row whose first halves would otherwise fill only the even 16-B bank slots
// (2-way conflicts: 2.5 extra cycles per LDS instruction measured on the
// 3B preset).
template <int D>
__device__ __forceinline__ int vswz(int r) {
    if constexpr (D == 64)
        return 2 * (r & 1) + 4 * ((r >> 1) & 3);
    else
        return 4 * (r & 7);
}

// physical quad of logical quad q of row r
template <int D>
__device__ __forceinline__ int vquad(int r, int q) {
    const int t = q ^ vswz<D>(r);
    if constexpr (D == 128)
        return t ^ (2 * ((t >> 4) & 1));
    else
        return t;
}

// One tile of the MFMA per-row kernel: V -> the wave's LDS tile, S^T on the
// matrix cores, then (prefetch) the tile two ahead is loaded into the same
// registers while the softmax and the PV product run.
template <int D, bool KV8>
__device__ __forceinline__ void attn_tile_mfma(KVTile<D, KV8>& cur, bool prefetch, int kt_next, const KVSrc& src,
                                               int kt, int end, int lane, int g16, uint16_t* vw,
                                               const uint16_t* tr0, int trk, int tr_half,
                                               const bf16x8_t (&qf)[D / 32], float& m, float& l,
                                               f32x4_t (&acc)[D / 16], float scale_log2) {
    constexpr int KS = D / 32;
    constexpr int DB = D / 16;
    const bool partial = kt + 32 > end;
    if constexpr (KV8) {  // 16 e4m3 per chunk -> two 8-bf16 LDS stores (quads q, q+2)
        constexpr int CPK = D / 16;
#pragma unroll
        for (int r = 0; r < D / 32; ++r) {
            const int ch = lane + kWave * r;
            const int row = ch / CPK, q = 4 * (ch % CPK);
            uint16_t* rp = vw + row * D;
            *reinterpret_cast<uint4*>(rp + 4 * vquad<D>(row, q)) = fp8x8_to_bf16x8(make_uint2(cur.v[r].x, cur.v[r].y));
            *reinterpret_cast<uint4*>(rp + 4 * vquad<D>(row, q + 2)) =
                fp8x8_to_bf16x8(make_uint2(cur.v[r].z, cur.v[r].w));
        }
    } else {
        constexpr int CPK = D / 8;
#pragma unroll
        for (int r = 0; r < D / 16; ++r) {
            const int ch = lane + kWave * r;
            const int row = ch / CPK;
            *reinterpret_cast<uint4*>(vw + row * D + 4 * vquad<D>(row, 2 * (ch % CPK))) = cur.v[r];
        }
    }
    f32x4_t sacc[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        sacc[h] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            bf16x8_t kf;
            if constexpr (KV8)
                kf = as_bf16x8(fp8x8_to_bf16x8(cur.k[h][ks]));
            else
                kf = as_bf16x8(cur.k[h][ks]);
            sacc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], sacc[h], 0, 0, 0);
        }
    }
    if (prefetch) load_kv_tile<D, KV8>(src, kt_next, end, lane, cur);
    // S^T tile: register 4h+i = key kt + 16h + 4*g16 + i of query (lane&15).
    // Scale folded into one FMA per score; the key mask only on a partial
    // last tile; hardware exp2 and bf16 packing.
    float tmax = -1e30f;
    if (!partial) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i) tmax = fmaxf(tmax, sacc[h][i]);
    } else {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int key = kt + 16 * h + 4 * g16 + i;
                sacc[h][i] = key < end ? sacc[h][i] : -1e30f;
                tmax = fmaxf(tmax, sacc[h][i]);
            }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, kWave));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, kWave)) * scale_log2;
    const float mn = fmaxf(m, tmax);
    if (__any(mn > m)) {
        const float corr = __builtin_amdgcn_exp2f(m - mn);
        l *= corr;
#pragma unroll
        for (int db = 0; db < DB; ++db) acc[db] *= corr;
    }
    m = mn;
    f32x8_t pr;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            pr[4 * h + i] = __builtin_amdgcn_exp2f(fmaf(sacc[h][i], scale_log2, -mn));
            l += pr[4 * h + i];  // lane-partial sum; the 4 groups are added once at the end
        }
    // B operand P^T: element j = key pi(8*g16 + j) = 16*(j>>2) + 4*g16 + (j&3)
    const bf16x8_t pf = __builtin_convertvector(pr, bf16x8_t);
#pragma unroll
    for (int db = 0; db < DB; ++db) {
        // the two transposed reads (keys +0 / +16) as whole 32-bit registers;
        // d block db sits at quad group db ^ trk of the lane's swizzled row
        // (D = 128: halves swapped in groups with bit 2 set, see vquad)
        const int grp = db ^ trk;
        const uint16_t* tp = tr0 + 16 * grp;
        if constexpr (D == 128) tp += ((grp >> 2) & 1) * tr_half;
        const uint2 lo = __builtin_bit_cast(
            uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16_t*)tp));
        const uint2 hi = __builtin_bit_cast(
            uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16_t*)(tp + 16 * D)));
        const uint4 a = make_uint4(lo.x, lo.y, hi.x, hi.y);
        acc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a), pf, acc[db], 0, 0, 0);
    }
}

// --------------------------------------------------------------------------
// 3c. per-row decode attention on the matrix cores.
//    Writes split partials at index ps_max + split (the shared prefix's
//    partials take [0, ps_max)) for the combine kernel, ONE WAVE per work item
//    (row, kv head, split) and both products on MFMA 16x16x32 bf16 per
//    32-key tile:
//        S^T[key, q] = K[key, :] . Q^T[:, q]      A = K rows straight from HBM
//                                                  (16 B per lane), B = Q^T
//        O^T[d, q]  += V^T[d, key] . P^T[key, q]  A = V^T read transposed out
//                                                  of the wave's LDS tile with
//                                                  ds_read_b64_tr_b16, B = P^T
//    The G query heads of the kv head are the MFMA's N columns (padded to
//    16).  S^T leaves the query on the lane and 8 keys in registers, so the
//    online softmax is in-register + 2 cross-group shuffles per tile, and P^T
//    is the PV B operand with no data movement: the PV k order is the
//    permutation {4g..4g+3, 16+4g..16+4g+3} of lane group g, matched by the
//    two transposed V reads (rows 4g.. and 16+4g..).
//    The kernel is bound by HBM latency x bytes in flight, not by math
//    (profiles/decode_step_*: a 1-deep prefetch with 1024-key splits ran at
//    42 % of the copy rate): each row's keys are cut into equal splits sized
//    so that ~16 waves per CU are busy, and each wave keeps the next tile's
//    K/V loads in flight while it computes the current one.  (A register
//    double buffer of two tiles in flight measured no faster; removed.)
//    Measured and not adopted (profiles/decode_step_r2_notes.md): merging a
//    sequence's jump-forward rows into one work item (their keys read once)
//    gained nothing -- those re-reads already hit L2 / MALL -- and its extra
//    per-item work cost 2 %; a branch-free steady-state loop cut VALU
//    instructions per tile but not time (the kernel waits on memory).
//    No block-level synchronisation: each wave owns its LDS tile, so
//    different waves of a block run different items.
// --------------------------------------------------------------------------
template <int D, bool KV8>
__global__ __launch_bounds__(kBlock) void decode_attn_mfma_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ k_cache, const void* __restrict__ v_cache,
    const int32_t* __restrict__ slot, const int32_t* __restrict__ seq_len, uint16_t* __restrict__ out,
    float* __restrict__ part_o, float* __restrict__ part_ml, int B, int Hkv, int G,
    int max_seq, int chunk, int splits, float scale_log2, int num_slots, const int32_t* __restrict__ plen,
    int ps_max, const int32_t* __restrict__ prow, const int32_t* __restrict__ fork) {
    static_assert(D % 32 == 0, "D must be a multiple of 32");
    constexpr int KS = D / 32;    // 32-dim k-steps of the S product
    constexpr int DB = D / 16;    // 16-row d blocks of O^T
    constexpr int NW = kBlock / kWave;
    __shared__ __attribute__((aligned(16))) uint16_t vlds[NW][32 * D];
    const int lane = threadIdx.x & (kWave - 1);
    // wave index made provably uniform: the item loop, its bounds and the
    // slot / seq_len reads stay scalar (no exec-masked control flow, which
    // ds_read_b64_tr_b16 must not run under, and no scratch)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int g16 = lane >> 4, c = lane & 15;
    const int Hq = Hkv * G;
    const int P0 = __builtin_amdgcn_readfirstlane(plen ? max(0, *plen) : 0);
    const int splits_total = ps_max + splits;
    const int total = B * Hkv * splits;
    uint16_t* vw = vlds[wave];
    // transposed-read addresses (tile-invariant): lane 4q+p of group g16 reads
    // row 4*g16 + q (and 16 + ...), columns 4p..4p+3 of each 16-wide d block,
    // through the row's swizzle (vswz)
    const int trow = 4 * g16 + (c >> 2), tsw = vswz<D>(trow);
    const uint16_t* tr0 = vw + trow * D + 4 * ((c & 3) ^ (tsw & 3));
    const int trk = tsw >> 2;
    // D = 128 swapped halves: quad p ^ 2 of the group, as an element offset
    const int tr_half = (c & 2) ? -8 : 8;
    for (int item = blockIdx.x * NW + wave; item < total; item += gridDim.x * NW) {
        // split-major: consecutive waves take different rows' splits, so the
        // persistent grid's first pass covers every row; inside a split kv
        // head-major, so a block's 4 waves take 4 consecutive rows of one kv
        // head -- a slot's jump-forward rows (consecutive rows, the same keys)
        // re-read them on one CU / XCD instead of from the MALL
        const int split = item / (B * Hkv);
        const int rem = item - split * (B * Hkv);
        const int kh = rem / B, b = rem - kh * B;
        const int s = __builtin_amdgcn_readfirstlane(slot[b]);
        const int L = __builtin_amdgcn_readfirstlane((s >= 0 && s < num_slots) ? min(seq_len[b], max_seq) : 0);
        if (L <= 0) {  // padding row / bad slot: defined output, nothing read
            if (split == 0)
                for (int o = lane; o < G * D; o += kWave) out[((size_t)b * Hq + kh * G) * D + o] = 0;
            continue;
        }
        // a row outside the shared prefix (prow[b] == 0) owns all its keys
        const int P = __builtin_amdgcn_readfirstlane((prow && !prow[b]) ? 0 : P0);
        const SplitGeom sg = split_geom(L - P, splits, chunk);
        if (split >= max(1, sg.nact)) continue;
        // one own split: this wave writes the row's final output -- directly,
        // or (shared prefix) after merging the prefix kernel's partials, which
        // the same stream finished before this launch (no combine pass)
        const bool direct = P == 0 && sg.nact == 1;
        const bool merge_prefix = P > 0 && sg.nact <= 1;
        const int start = P + split * sg.part;
        const int end = min(L, start + sg.part);
        const int ntiles = (end - start + 31) / 32;
        bf16x8_t qf[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (c < G) v = *reinterpret_cast<const uint4*>(q + ((size_t)b * Hq + kh * G + c) * D + 32 * ks + 8 * g16);
            qf[ks] = as_bf16x8(v);
        }
        const size_t head_off = ((size_t)s * Hkv + kh) * (size_t)max_seq * D;
        KVSrc src{kv_at<KV8>(k_cache, head_off), kv_at<KV8>(v_cache, head_off), nullptr, nullptr, 0};
        if (fork) {  // fork[2 s] = parent slot, fork[2 s + 1] = the end of the shared keys
            const int ps = __builtin_amdgcn_readfirstlane(fork[2 * s]);
            const int fe = __builtin_amdgcn_readfirstlane(fork[2 * s + 1]);
            if (fe > 0 && ps >= 0 && ps < num_slots && ps != s) {
                const size_t poff = ((size_t)ps * Hkv + kh) * (size_t)max_seq * D;
                src.pk = kv_at<KV8>(k_cache, poff);
                src.pv = kv_at<KV8>(v_cache, poff);
                src.fend = min(fe, L);
            }
        }
        float m = -1e30f, l = 0.f;
        f32x4_t acc[DB];
#pragma unroll
        for (int db = 0; db < DB; ++db) acc[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        KVTile<D, KV8> ta;
        load_kv_tile<D, KV8>(src, start, end, lane, ta);
        for (int t = 0; t < ntiles; ++t) {
            const int kt = start + 32 * t;
            attn_tile_mfma<D, KV8>(ta, t + 1 < ntiles, kt + 32, src, kt, end, lane, g16, vw, tr0, trk, tr_half, qf, m, l,
                                   acc, scale_log2);
        }
        l += __shfl_xor(l, 16, kWave);
        l += __shfl_xor(l, 32, kWave);
        if (c < G && merge_prefix) {
            const int qh = kh * G + c;
            const size_t pb = ((size_t)b * Hq + qh) * splits_total;
            // online log-sum-exp merge of the ps_max prefix partials into
            // this wave's (m, l, acc) -- the combine kernel's arithmetic
            for (int sp = 0; sp < ps_max; ++sp) {
                const float2 ml = *reinterpret_cast<const float2*>(part_ml + (pb + sp) * 2);
                const float mn = fmaxf(m, ml.x);
                const float ca = __builtin_amdgcn_exp2f(m - mn), cb = __builtin_amdgcn_exp2f(ml.x - mn);
                l = l * ca + ml.y * cb;
#pragma unroll
                for (int db = 0; db < DB; ++db) {
                    const float4 o = *reinterpret_cast<const float4*>(part_o + (pb + sp) * D + 16 * db + 4 * g16);
                    acc[db][0] = acc[db][0] * ca + o.x * cb;
                    acc[db][1] = acc[db][1] * ca + o.y * cb;
                    acc[db][2] = acc[db][2] * ca + o.z * cb;
                    acc[db][3] = acc[db][3] * ca + o.w * cb;
                }
                m = mn;
            }
            const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
            for (int db = 0; db < DB; ++db) {
                const float f[4] = {acc[db][0] * inv, acc[db][1] * inv, acc[db][2] * inv, acc[db][3] * inv};
                *reinterpret_cast<uint2*>(out + ((size_t)b * Hq + qh) * D + 16 * db + 4 * g16) = pack4(f);
            }
        } else if (c < G) {
            const int qh = kh * G + c;
            const float inv = l > 0.f ? 1.f / l : 0.f;
            const size_t pi = ((size_t)b * Hq + qh) * splits_total + ps_max + split;
#pragma unroll
            for (int db = 0; db < DB; ++db) {
                const int d0 = 16 * db + 4 * g16;
                if (direct) {
                    const float f[4] = {acc[db][0] * inv, acc[db][1] * inv, acc[db][2] * inv, acc[db][3] * inv};
                    *reinterpret_cast<uint2*>(out + ((size_t)b * Hq + qh) * D + d0) = pack4(f);
                } else {
                    *reinterpret_cast<float4*>(part_o + pi * D + d0) =
                        make_float4(acc[db][0], acc[db][1], acc[db][2], acc[db][3]);
                }
            }
            if (!direct && g16 == 0) {
                part_ml[pi * 2] = m;
                part_ml[pi * 2 + 1] = l;
            }
        }
    }
}

// CUs of the current device (cached per device; 256 on MI355X)
inline int device_cu_count() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cached[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev] = n;
    }
    return cached[dev];
}

inline int grid_for(size_t work) {
    size_t g = (work + kBlock - 1) / kBlock;
    if (g > 2048) g = 2048;  // grid-stride beyond 8 blocks/CU (Guideline 11)
    return (int)(g == 0 ? 1 : g);
}

hipError_t launch_combine(void* part_o, void* part_ml, const int32_t* sl, const int32_t* ln, void* out, int B, int Hq,
                          int D, int max_seq, int chunk, int splits, int num_slots, const int32_t* pl, int ps_max,
                          const int32_t* pr, hipStream_t st) {
    const int waves = B * Hq;
    const int blocks = (waves + 3) / 4;
    const dim3 grid((unsigned)(blocks < 2048 ? blocks : 2048));
    if (D == 64)
        decode_attn_combine_kernel<64><<<grid, kBlock, 0, st>>>((const float*)part_o, (const float*)part_ml, sl, ln,
                                                               (uint16_t*)out, B, Hq, max_seq, chunk, splits,
                                                               num_slots, pl, ps_max, pr);
    else if (D == 128)
        decode_attn_combine_kernel<128><<<grid, kBlock, 0, st>>>((const float*)part_o, (const float*)part_ml, sl, ln,
                                                                (uint16_t*)out, B, Hq, max_seq, chunk, splits,
                                                                num_slots, pl, ps_max, pr);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace

// ---- method-branch KV fork: slot src's keys and values at positions
// [start, end) of every layer and kv head into up to 32 destination slots,
// one launch for both caches (LocalLM.fork_kv; it replaced two indexed-copy
// launches per fork).  Caches [layers][slots][Hkv][max_seq][row_bytes];
// each thread moves 16 B: read once, written ndst times.
struct ForkDsts {
    int32_t d[32];
};

__global__ __launch_bounds__(kBlock) void kv_fork_kernel(uint8_t* __restrict__ kc, uint8_t* __restrict__ vc,
                                                         int layers, int num_slots, int Hkv, int max_seq,
                                                         int row_bytes, int src, ForkDsts dsts, int ndst, int start,
                                                         int span16) {
    // span16: 16-B units of one (layer, head) run = (end - start) * row_bytes / 16
    const long per_cache = (long)layers * Hkv * span16;
    const long total = 2 * per_cache;
    for (long u = (long)blockIdx.x * kBlock + threadIdx.x; u < total; u += (long)gridDim.x * kBlock) {
        const bool isv = u >= per_cache;
        const long w = isv ? u - per_cache : u;
        const int lh = (int)(w / span16), off = (int)(w - (long)lh * span16);
        const int layer = lh / Hkv, h = lh - layer * Hkv;
        uint8_t* base = isv ? vc : kc;
        const size_t run = (size_t)start * row_bytes + (size_t)off * 16;
        auto at = [&](int slot) -> uint4* {
            return reinterpret_cast<uint4*>(
                base + ((((size_t)layer * num_slots + slot) * Hkv + h) * (size_t)max_seq) * row_bytes + run);
        };
        const uint4 v = *at(src);
        for (int i = 0; i < ndst; ++i) *at(dsts.d[i]) = v;
    }
}

extern "C" {

int dmcp_abi_version() { return 17; }

int dmcp_add_rmsnorm(const void* x, void* residual, const void* w, void* out, int rows, int H, float eps,
                     void* stream) {
    if (H % 8 != 0 || H > kBlock * 8 * 4 || rows <= 0) return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    const int vpt = (H + kBlock * 8 - 1) / (kBlock * 8);
    auto xx = (const uint16_t*)x;
    auto rr = (uint16_t*)residual;
    auto ww = (const uint16_t*)w;
    auto oo = (uint16_t*)out;
    if (vpt == 1) add_rmsnorm_kernel<1><<<rows, kBlock, 0, st>>>(xx, rr, ww, oo, H, eps);
    else if (vpt == 2) add_rmsnorm_kernel<2><<<rows, kBlock, 0, st>>>(xx, rr, ww, oo, H, eps);
    else add_rmsnorm_kernel<4><<<rows, kBlock, 0, st>>>(xx, rr, ww, oo, H, eps);
    return hipGetLastError();
}

int dmcp_rope_kv(const void* qkv, const void* pos, const void* slot, const void* cos_sin, void* q_out,
                 void* k_cache, void* v_cache, int T, int Hq, int Hkv, int D, int max_seq, int max_pos,
                 int num_slots, int kv8, void* stream) {
    if (T <= 0) return 0;
    if (D % 16 != 0) return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    if (kv8)
        rope_kv_kernel<true><<<T, kBlock, 0, st>>>((const uint16_t*)qkv, (const int32_t*)pos, (const int32_t*)slot,
                                                   (const float2*)cos_sin, (uint16_t*)q_out, k_cache, v_cache, Hq,
                                                   Hkv, D, max_seq, max_pos, num_slots);
    else
        rope_kv_kernel<false><<<T, kBlock, 0, st>>>((const uint16_t*)qkv, (const int32_t*)pos, (const int32_t*)slot,
                                                    (const float2*)cos_sin, (uint16_t*)q_out, k_cache, v_cache, Hq,
                                                    Hkv, D, max_seq, max_pos, num_slots);
    return hipGetLastError();
}

// q [B, Hq, D]; caches [S, Hkv, max_seq, D] (bf16, or fp8 e4m3 with kv8);
// slot / seq_len [B].  With plen: every row's first *plen keys are the shared
// prefix in prefix_k / prefix_v ([Hkv, max_seq, D], the prefix slot), read by
// the MFMA prefill kernel in prefix mode into ps_max partials per row; the
// per-row kernel covers keys [*plen, L).  Partials of both are merged by the
// combine kernel; a row that fits one split with no prefix is written directly.
// prefix_rows (optional, int32 [B]): 0 marks a row that does not use the
// shared prefix (its keys [0, L) are all in its own slot).
int dmcp_decode_attention(const void* q, const void* k_cache, const void* v_cache, const void* slot,
                          const void* seq_len, void* out, void* part_o, void* part_ml, int B, int Hq, int Hkv, int D,
                          int max_seq, int num_slots, int chunk, int splits, float scale, const void* prefix_k,
                          const void* prefix_v, const void* plen, int ps_max, int kv8, const void* prefix_rows,
                          const void* fork, void* stream) {
    if (B <= 0) return 0;
    if (Hkv <= 0 || Hq % Hkv != 0 || splits <= 0 || chunk <= 0 || !(D == 64 || D == 128) || Hq / Hkv > 16)
        return hipErrorInvalidValue;
    const bool prefix = plen != nullptr;
    if (prefix && (!prefix_k || !prefix_v || ps_max <= 0)) return hipErrorInvalidValue;
    if (!prefix) ps_max = 0;
    if ((splits > 1 || prefix) && (!part_o || !part_ml)) return hipErrorInvalidValue;
    const int G = Hq / Hkv;
    const float sl2 = scale * 1.4426950408889634f;
    auto st = (hipStream_t)stream;
    auto qq = (const uint16_t*)q;
    auto sl = (const int32_t*)slot;
    auto ln = (const int32_t*)seq_len;
    auto pl = (const int32_t*)plen;
    auto pr = prefix ? (const int32_t*)prefix_rows : nullptr;
    if (prefix) {
        hipError_t pe = dmcp_launch_prefix_partials(qq, prefix_k, prefix_v, pl, (float*)part_o, (float*)part_ml, B,
                                                    Hkv, G, D, max_seq, ps_max, ps_max + splits, sl2, kv8, st);
        if (pe != hipSuccess) return pe;
    }
    // persistent grid: one wave per (split, row, kv head) item, a block runs
    // 4; as many blocks as are resident at once (the kernel's occupancy: 4
    // per CU at D = 64, 2-3 at D = 128), never more than items -- a grid past
    // residency runs a trailing partial round
    const long items = (long)splits * Hkv * B;
    const long wblocks = (items + 3) / 4;
    float* po = (float*)part_o;
    float* pml = (float*)part_ml;
    uint16_t* oo = (uint16_t*)out;
#define DMCP_MFMA_DECODE(DD, K8)                                                                                   \
    do {                                                                                                           \
        static int per_cu = 0;                                                                                     \
        if (per_cu <= 0 && (hipOccupancyMaxActiveBlocksPerMultiprocessor(                                         \
                                &per_cu, decode_attn_mfma_kernel<DD, K8>, kBlock, 0) != hipSuccess ||           \
                            per_cu <= 0))                                                                          \
            per_cu = 4;                                                                                            \
        const long cap = (long)per_cu * device_cu_count();                                                         \
        const dim3 wgrid((unsigned)(wblocks < cap ? wblocks : cap));                                               \
        decode_attn_mfma_kernel<DD, K8><<<wgrid, kBlock, 0, st>>>(qq, k_cache, v_cache, sl, ln, oo, po, pml, B,   \
                                                                  Hkv, G, max_seq, chunk, splits, sl2, num_slots, \
                                                                  pl, ps_max, pr, (const int32_t*)fork);          \
    } while (0)
    if (kv8) {
        if (D == 64) DMCP_MFMA_DECODE(64, true);
        else DMCP_MFMA_DECODE(128, true);
    } else {
        if (D == 64) DMCP_MFMA_DECODE(64, false);
        else DMCP_MFMA_DECODE(128, false);
    }
#undef DMCP_MFMA_DECODE
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || splits == 1) return e;  // every row finished in the main kernel
    return launch_combine(part_o, part_ml, sl, ln, out, B, Hq, D, max_seq, chunk, splits, num_slots, pl, ps_max, pr,
                          st);
}

int dmcp_silu_mul(const void* gu, void* out, int T, int I, void* stream) {
    if (I % 8 != 0) return hipErrorInvalidValue;
    if (T <= 0) return 0;
    silu_mul_kernel<<<grid_for((size_t)T * (I / 8)), kBlock, 0, (hipStream_t)stream>>>((const uint16_t*)gu,
                                                                                      (uint16_t*)out, T, I);
    return hipGetLastError();
}

int dmcp_masked_argmax(const void* logits, const void* mask, const void* mask_idx, int n_masks, void* ids, int B,
                       int V, int ld, void* stream) {
    if (B <= 0) return 0;
    if (mask_idx && n_masks <= 0) return hipErrorInvalidValue;
    // whole 16-B chunks only when every row start is 16-B aligned
    const bool vec = (ld % 8 == 0) && (reinterpret_cast<uintptr_t>(logits) % 16 == 0);
    masked_argmax_kernel<<<B, MA_T, 0, (hipStream_t)stream>>>((const uint16_t*)logits, (const uint32_t*)mask,
                                                             (const int32_t*)mask_idx, n_masks, (int32_t*)ids, V,
                                                             ld, vec ? V / 8 : 0);
    return hipGetLastError();
}

int dmcp_decode_embed_norm(const void* table, const void* tokens, const void* src, const void* last_ids,
                           const void* pos, const void* w, void* resid, void* h, void* seq_len, int rows, int H,
                           int V, int n_last, float eps, void* mask_idx, const void* mask_alt, int alt_token,
                           void* stream) {
    if (H % 8 != 0 || H > kBlock * 8 * 4 || V <= 0 || (src && (!last_ids || n_last <= 0)) || (h && !w) ||
        (mask_alt && (!mask_idx || !src)))
        return hipErrorInvalidValue;
    if (rows <= 0) return 0;
    auto st = (hipStream_t)stream;
    const int vpt = (H + kBlock * 8 - 1) / (kBlock * 8);
    auto args = [&](auto kern) {
        kern<<<rows, kBlock, 0, st>>>((const uint16_t*)table, (const int32_t*)tokens, (const int32_t*)src,
                                      (const int32_t*)last_ids, (const int32_t*)pos, (const uint16_t*)w,
                                      (uint16_t*)resid, (uint16_t*)h, (int32_t*)seq_len, H, V, n_last, eps,
                                      (int32_t*)mask_idx, (const int32_t*)mask_alt, alt_token);
    };
    if (vpt == 1) args(decode_embed_norm_kernel<1>);
    else if (vpt == 2) args(decode_embed_norm_kernel<2>);
    else args(decode_embed_norm_kernel<4>);
    return hipGetLastError();
}

int dmcp_embedding(const void* table, const void* ids, void* out, int T, int H, int V, void* stream) {
    if (H % 8 != 0) return hipErrorInvalidValue;
    if (T <= 0) return 0;
    embedding_kernel<<<grid_for((size_t)T * (H / 8)), kBlock, 0, (hipStream_t)stream>>>(
        (const uint16_t*)table, (const int32_t*)ids, (uint16_t*)out, T, H, V);
    return hipGetLastError();
}

// see kv_fork_kernel; row_bytes = head_dim x element size, a multiple of 16
int dmcp_kv_fork(void* k_cache, void* v_cache, int layers, int num_slots, int Hkv, int max_seq, int row_bytes,
                 int src, const int32_t* dsts, int ndst, int start, int end, void* stream) {
    if (end <= start || ndst <= 0) return 0;
    if (!k_cache || !v_cache || row_bytes % 16 != 0 || ndst > 32 || src < 0 || src >= num_slots || start < 0 ||
        end > max_seq)
        return hipErrorInvalidValue;
    ForkDsts d{};
    for (int i = 0; i < ndst; ++i) {
        if (dsts[i] < 0 || dsts[i] >= num_slots) return hipErrorInvalidValue;
        d.d[i] = dsts[i];
    }
    const int span16 = (int)((size_t)(end - start) * row_bytes / 16);
    const long total = 2L * layers * Hkv * span16;
    const int grid = (int)std::min<long>((total + kBlock - 1) / kBlock, 4096);
    kv_fork_kernel<<<grid, kBlock, 0, (hipStream_t)stream>>>((uint8_t*)k_cache, (uint8_t*)v_cache, layers, num_slots,
                                                             Hkv, max_seq, row_bytes, src, d, ndst, start, span16);
    return hipGetLastError();
}

}  // extern "C"
