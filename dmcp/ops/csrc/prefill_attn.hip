// Flash-style prefill / extend attention for gfx950 (MI355X, CDNA4) -- the
// attention of one sequence's T new tokens (positions [start, start+T)) over
// every key at or before each token, in ONE pass on the matrix cores:
//
//   * keys [0, P) come from the shared-prefix slot (the enrichment prompt's
//     instructions + README, prefilled once per batch), keys [P, start+T)
//     from the sequence's own slot -- no per-sequence copy of the prefix, no
//     GQA head expansion, no two-kernel log-sum-exp merge (the SDPA path it
//     replaces: dmcp/models/llm.py::_extend_attention);
//   * causal masking only on the tiles that straddle a query's position.
//
// Formulation (the 'swapped QK^T' attention of cdna_hip_programming.md
// "Fused attention prefill"): per 32-key tile and 32 query columns
//     S^T[key, col] = K[key, :] . Q^T[:, col]          32x32x16 bf16, D/16 k-steps
//     O^T[d, col]  += V^T[d, key] . P^T[key, col]      32x32x16 bf16, 2 k-steps per d tile
// S^T lands with the query column on the lane and 16 keys in registers, so
// the online softmax is per lane (+ one cross-half shuffle) and P^T feeds the
// second product as its B operand in place (accumulator-as-operand idiom,
// permuted k order).  The V^T operand is read from a ROW-major V tile with
// the CDNA4 hardware transpose read ds_read_b64_tr_b16 (T10), so K and V are
// staged with plain 16-byte row copies.
//
// Query columns are (token, q head of the kv group) pairs flattened as
// token * G + g (any group size G).  A work item = (kv head, 32 * NSUB * 4
// columns): its 4 (or 8) waves each own NSUB 32-column units and share every K/V
// tile the block stages in LDS (64 keys per stage, two buffers, global loads
// for stage s+1 issued before stage s is computed and written after it --
// the register-staged pipeline of T14).  Block b takes kv head b % Hkv, so
// with Hkv = 8 each XCD's L2 holds one head's K/V; heavy (late, more keys)
// column tiles are dispatched first.
//
// LDS image: [64 keys][D] bf16 rows with the 16-byte chunk index XOR-swizzled
// per row (pf_swz) so that both the K row reads (ds_read_b128, lane = key)
// and the V transposed reads (4 rows x 16 columns per 16-lane group) are
// bank-conflict free for D = 64 (derivation in pf_swz); D = 128 uses the
// guide's 256-B-row swizzle.
#include "dmcp_common.hpp"

namespace {

constexpr int kPfKeys = 64;  // keys per LDS stage (two 32-key MFMA tiles)
constexpr float kRescaleSlack = 8.f;  // deferred online-softmax rescale threshold (log2 units)

// chunk swizzle of row `row`:
//  D = 64 (8 chunks, 128-B rows: two rows per 256-B bank line).  With
//  e = row >> 1, f(e) = ((e & 1) << 2) | ((e >> 1) & 3):
//   - K row reads: each ds_read_b128 pass serves 16 lanes = 8 even + 8 odd
//     rows of {0-3,12-15,20-27} or {4-11,16-19,28-31}; f takes 8 distinct
//     values on each pass's even (and odd) rows -> 16 distinct 16-B slots;
//   - V transposed reads: a 32-lane half reads rows 4m..4m+3, chunks
//     4t..4t+3; rows 4m and 4m+2 differ in bit 2 of f, so their chunks land
//     in different 4-chunk halves of the bank line (likewise 4m+1 / 4m+3).
//  D = 128: (row & 3) << 2 | (row >> 2) & 3 (cdna_hip_programming.md T10 (b)).
template <int D>
__device__ __forceinline__ int pf_swz(int row) {
    if constexpr (D == 64)
        return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
    else
        return ((row & 3) << 2) | ((row >> 2) & 3);
}

template <int D>
__device__ __forceinline__ int pf_off(int row, int ch) {
    return row * D + 8 * (ch ^ pf_swz<D>(row));
}

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses row q,
// columns 4p..4p+3 of a 4 x 16 block; lane i receives column i (row q in
// element q).  EXEC must be full: callers never diverge around it.
__device__ __forceinline__ v4i16_t lds_tr16(const uint16_t* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16_t*)(p));
}

// The work of one block: kv head kh, column tile ct (32 * NSUB * NWAVE query
// columns), key split sp of nsplit.  Shared by the single-sequence kernel,
// the varlen (packed multi-sequence) kernel and the decode step's prefix mode.
template <int D, int NSUB, int NWAVE, bool KV8>
__device__ __forceinline__ void prefill_attn_block(
    const uint16_t* __restrict__ q, const void* __restrict__ kc, const void* __restrict__ vc,
    const void* __restrict__ pk, const void* __restrict__ pv, uint16_t* __restrict__ out,
    float* __restrict__ part_o, float* __restrict__ part_ml, int T, int start, int P, int Hkv, int G, int ldk,
    int kh, int sp, int ct, int nsplit, float sl2, const int32_t* __restrict__ plen, long prs, long pss) {
    constexpr int KS = D / 16;  // k-steps of the QK product
    constexpr int DT = D / 32;  // 32-row d tiles of the PV product
    constexpr int CH = D / 8;   // 16-byte chunks per row
    constexpr int NT = NWAVE * kWave;
    constexpr int COLS = 32 * NSUB * NWAVE;
    constexpr int LU = (kPfKeys * CH + NT - 1) / NT;  // 16-B loads per thread per stage (K and V each)
    static_assert(kPfKeys * CH % NT == 0, "stage must split evenly over the block");
    __shared__ __attribute__((aligned(16))) uint16_t sK[2][kPfKeys * D];
    __shared__ __attribute__((aligned(16))) uint16_t sV[2][kPfKeys * D];

    const int Hq = Hkv * G;
    const int NC = T * G;
    const int c0 = ct * COLS;
    // prefix mode (plen != nullptr, the decode step's shared prefix): every
    // query sees keys [0, *plen) -- read in the kernel so a captured graph
    // follows prefix changes -- all from pk/pv, and the output is always
    // partials (merged with the rows' own keys by decode_attn_combine_kernel)
    const bool prefix_mode = plen != nullptr;
    int kend;
    if (prefix_mode) {
        kend = __builtin_amdgcn_readfirstlane(max(0, min(*plen, ldk)));
        P = kend;
    } else {
        kend = start + (min(NC, c0 + COLS) - 1) / G + 1;  // keys [0, kend) are visible to the block
    }
    const int nst_all = (kend + kPfKeys - 1) / kPfKeys;
    // split-K: this block's stages [st0, st1) of the column tile's key range
    const int per = (nst_all + nsplit - 1) / nsplit;
    const int st0 = min(nst_all, sp * per), st1 = min(nst_all, st0 + per);
    // the wave index through readfirstlane: every per-unit bound below is then
    // provably wave-uniform, so the tile-skip and mask decisions compile to
    // scalar branches instead of exec-mask save/restore sequences
    const int lane = threadIdx.x & (kWave - 1), wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int r = lane & 31, h = lane >> 5;

    int qpos[NSUB], qmin[NSUB], qmax[NSUB], cf[NSUB];
    bool uact[NSUB];
    bf16x8_t qf[NSUB][KS];
    f32x16_t o[NSUB][DT];
    float m[NSUB], l[NSUB];
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
        cf[u] = c0 + (wave * NSUB + u) * 32;
        uact[u] = cf[u] < NC;
        const int cl = min(cf[u] + 31, NC - 1);
        qmin[u] = start + cf[u] / G;
        qmax[u] = start + cl / G;
        const int c = min(cf[u] + r, NC - 1);  // padding lanes repeat the last column; results discarded
        const int t = c / G, g = c - t * G;
        qpos[u] = start + t;
        const uint16_t* qp = q + ((size_t)t * Hq + (size_t)kh * G + g) * D + 8 * h;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            qf[u][ks] = as_bf16x8(*reinterpret_cast<const uint4*>(qp + 16 * ks));
            // re-define the Q registers here (an empty asm "writing" them): the
            // waitcnt pass otherwise carried the Q loads' scores around the key
            // loop and made the QK^T MFMAs wait vmcnt(3..0) on each stage's
            // K/V prefetch
            asm volatile("" : "+v"(qf[u][ks]));
        }
        m[u] = -1e30f;  // finite; kept equal across the two lane halves; l is per half
        l[u] = 0.f;
#pragma unroll
        for (int t2 = 0; t2 < DT; ++t2)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[u][t2][i] = 0.f;
    }

    // register-staged K/V tiles, held RAW while in flight (fp8 caches are
    // widened to bf16 only in store(), after the stage's compute: converting
    // at the load made every prefetch wait for its own data -- vmcnt(0) right
    // behind each load -- so nothing was in flight while a stage computed).
    // Rows past kend re-read row kend - 1 (a written row: finite), never
    // visible -- every such key is masked to -inf, so its P is 0.
    using Raw = std::conditional_t<KV8, uint2, uint4>;
    Raw kx[LU], vx[LU];
    auto load = [&](int st) {
#pragma unroll
        for (int i = 0; i < LU; ++i) {
            const int idx = threadIdx.x + i * NT;
            const int row = idx / CH, ch = idx - row * CH;
            const int key = min(st * kPfKeys + row, kend - 1);
            const bool pre = key < P;
            const size_t off = ((size_t)kh * ldk + key) * D + ch * 8;
            kx[i] = *reinterpret_cast<const Raw*>(kv_ptr<KV8>(pre ? pk : kc, off));
            vx[i] = *reinterpret_cast<const Raw*>(kv_ptr<KV8>(pre ? pv : vc, off));
        }
    };
    auto widen = [&](const Raw& v) -> uint4 {
        if constexpr (KV8)
            return fp8x8_to_bf16x8(v);
        else
            return v;
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < LU; ++i) {
            const int idx = threadIdx.x + i * NT;
            const int row = idx / CH, ch = idx - row * CH;
            *reinterpret_cast<uint4*>(&sK[buf][pf_off<D>(row, ch)]) = widen(kx[i]);
            *reinterpret_cast<uint4*>(&sV[buf][pf_off<D>(row, ch)]) = widen(vx[i]);
        }
    };

    if (st0 < st1) {
        load(st0);
        store(st0 & 1);
    }
    __syncthreads();
    // transposed-read lane geometry (see lds_tr16)
    const int i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3, g4 = lane >> 4;
    for (int st = st0; st < st1; ++st) {
        const int buf = st & 1;
        const bool more = st + 1 < st1;
        // the next stage's loads go out after the first tile's QK^T MFMAs
        // (in flight through the softmax / PV and the second tile): issued
        // ahead of them, their address registers were reused by the MFMA
        // destinations and every QK^T MFMA waited on vmcnt
        bool issued = !more;
        const uint16_t* Kt = sK[buf];
        const uint16_t* Vt = sV[buf];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            const int kb = st * kPfKeys + sub * 32;  // first key of this 32-key tile
            bool act[NSUB];
            bool any = false;
#pragma unroll
            for (int u = 0; u < NSUB; ++u) {
                act[u] = uact[u] && kb <= qmax[u];
                any |= act[u];
            }
            if (!any) continue;  // wave-uniform
            f32x16_t s[NSUB];
#pragma unroll
            for (int u = 0; u < NSUB; ++u)
#pragma unroll
                for (int i = 0; i < 16; ++i) s[u][i] = 0.f;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const bf16x8_t kf =
                    as_bf16x8(*reinterpret_cast<const uint4*>(Kt + pf_off<D>(sub * 32 + r, 2 * ks + h)));
#pragma unroll
                for (int u = 0; u < NSUB; ++u)
                    if (act[u]) s[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[u][ks], s[u], 0, 0, 0);
            }
            if (!issued) {
                load(st + 1);
                issued = true;
            }
            // online softmax; register i holds key kb + (i&3) + 8*(i>>2) + 4*h
            bf16x8_t pb[NSUB][2];
#pragma unroll
            for (int u = 0; u < NSUB; ++u) {
                if (!act[u]) continue;
                float mt = -1e30f;
                // mask: the tile straddles some query's position (causal) or
                // the end of the visible keys (prefix mode: no causal bound)
                if (kb + 31 > qmin[u] || kb + 32 > kend) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int key = kb + (i & 3) + 8 * (i >> 2) + 4 * h;
                        s[u][i] = (key <= qpos[u] && key < kend) ? s[u][i] : -INFINITY;
                        mt = fmaxf(mt, s[u][i]);
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) mt = fmaxf(mt, s[u][i]);
                }
                // masked scores are -inf and m starts at a finite -1e30, so a
                // lane with no visible key in the tile (or split) adds
                // exp2(-inf) = 0 and every rescale factor stays finite
                mt = half_swap_max(mt) * sl2;
                // deferred rescale (cdna_hip_programming.md "defer-max"): the
                // running max moves only when a tile max passes it by
                // kRescaleSlack (log2 units), so most tiles skip the O / l
                // rescale; P = exp2(s - m) stays <= 2^slack (exact in fp32
                // accumulators, bf16 P keeps its relative precision).  The
                // decision is wave-uniform and made before this tile's P.
                if (__any(mt > m[u] + kRescaleSlack)) {
                    const float mn = fmaxf(m[u], mt);
                    const float corr = __builtin_amdgcn_exp2f(m[u] - mn);
                    l[u] *= corr;
#pragma unroll
                    for (int t2 = 0; t2 < DT; ++t2)
#pragma unroll
                        for (int i = 0; i < 16; ++i) o[u][t2][i] *= corr;
                    m[u] = mn;
                }
                const float mn = m[u];
                f32x8_t p0, p1;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    p0[i] = __builtin_amdgcn_exp2f(fmaf(s[u][i], sl2, -mn));
                    p1[i] = __builtin_amdgcn_exp2f(fmaf(s[u][i + 8], sl2, -mn));
                    l[u] += p0[i] + p1[i];
                }
                pb[u][0] = __builtin_convertvector(p0, bf16x8_t);
                pb[u][1] = __builtin_convertvector(p1, bf16x8_t);
            }
            // O^T += V^T . P^T: V^T fragment element j of half h = key
            // 16*s2 + 8*(j>>2) + 4*h + (j&3) (P^T's register order), column d
#pragma unroll
            for (int t2 = 0; t2 < DT; ++t2) {
                const int ch = 4 * t2 + 2 * (g4 & 1) + (tp >> 1);
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int R0 = sub * 32 + 16 * s2 + 4 * h + tq;
                    // whole 32-bit registers of the two reads (a per-element
                    // 16-bit shuffle costs VALU and/or/shift packing per element)
                    const uint2 lo = __builtin_bit_cast(uint2, lds_tr16(Vt + pf_off<D>(R0, ch) + 4 * (tp & 1)));
                    const uint2 hi = __builtin_bit_cast(uint2, lds_tr16(Vt + pf_off<D>(R0 + 8, ch) + 4 * (tp & 1)));
                    const bf16x8_t vf = as_bf16x8(make_uint4(lo.x, lo.y, hi.x, hi.y));
#pragma unroll
                    for (int u = 0; u < NSUB; ++u)
                        if (act[u]) o[u][t2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb[u][s2], o[u][t2], 0, 0, 0);
                }
            }
        }
        if (!issued) load(st + 1);  // both tiles skipped (no query sees them)
        if (more) store(buf ^ 1);  // that buffer's readers finished before the last barrier
        __syncthreads();
    }

    // normalise and store: O^T register i of d tile t2 is d = 32*t2 + (i&3) + 8*(i>>2) + 4*h
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
        if (!uact[u]) continue;
        const float lt = half_swap_sum(l[u]);
        const int c = cf[u] + r;
        if (c >= NC) continue;
        const int t = c / G, g = c - t * G;
        const size_t row = (size_t)t * Hq + (size_t)kh * G + g;
        if (nsplit > 1 || prefix_mode) {  // unnormalised partial + (max, sum), merged by a combine kernel
            const size_t pr = (size_t)row * prs + (size_t)sp * pss;
            float* po = part_o + pr * D;
#pragma unroll
            for (int t2 = 0; t2 < DT; ++t2)
#pragma unroll
                for (int gi = 0; gi < 4; ++gi)
                    *reinterpret_cast<float4*>(po + 32 * t2 + 8 * gi + 4 * h) =
                        make_float4(o[u][t2][4 * gi], o[u][t2][4 * gi + 1], o[u][t2][4 * gi + 2], o[u][t2][4 * gi + 3]);
            if (h == 0) *reinterpret_cast<float2*>(part_ml + pr * 2) = make_float2(m[u], lt);
            continue;
        }
        const float inv = lt > 0.f ? 1.f / lt : 0.f;
        uint16_t* op = out + row * D;
#pragma unroll
        for (int t2 = 0; t2 < DT; ++t2)
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                const float f[4] = {o[u][t2][4 * gi] * inv, o[u][t2][4 * gi + 1] * inv, o[u][t2][4 * gi + 2] * inv,
                                    o[u][t2][4 * gi + 3] * inv};
                *reinterpret_cast<uint2*>(op + 32 * t2 + 8 * gi + 4 * h) = pack4(f);
            }
    }
}

template <int D, int NSUB, int NWAVE, bool KV8>
__global__ __launch_bounds__(NWAVE * 64) void prefill_attn_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ kc, const void* __restrict__ vc,
    const void* __restrict__ pk, const void* __restrict__ pv, uint16_t* __restrict__ out,
    float* __restrict__ part_o, float* __restrict__ part_ml, int T, int start, int P, int Hkv, int G, int ldk,
    int ctiles, int nsplit, float sl2, const int32_t* __restrict__ plen, long prs, long pss) {
    const int kh = blockIdx.x % Hkv;
    const int rest = (int)(blockIdx.x / Hkv);
    const int sp = rest % nsplit;
    const int ct = ctiles - 1 - rest / nsplit;  // heavy (late) column tiles first
    prefill_attn_block<D, NSUB, NWAVE, KV8>(q, kc, vc, pk, pv, out, part_o, part_ml, T, start, P, Hkv, G, ldk, kh, sp,
                                            ct, nsplit, sl2, plen, prs, pss);
}

// Packed multi-sequence prefill (the engine's batched admission): q / out
// [Ttot, Hq, D] hold every sequence's tokens back to back; block b runs work
// item b / Hkv of the host-built table (sequence, column tile), sorted by
// descending key count so the long tiles start first, for kv head b % Hkv.
// seq[i] = (token offset, T, start, slot, shared-prefix length).  No split-K:
// a batch of 2,000-token prompts is thousands of blocks already.
template <int D, int NSUB, int NWAVE, bool KV8>
__global__ __launch_bounds__(NWAVE * 64) void prefill_varlen_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ kcache, const void* __restrict__ vcache,
    const void* __restrict__ pk, const void* __restrict__ pv, uint16_t* __restrict__ out,
    const int32_t* __restrict__ items, const int32_t* __restrict__ seq, int Hkv, int G, int ldk, size_t slot_elems,
    float sl2) {
    const int kh = blockIdx.x % Hkv;
    const int it = blockIdx.x / Hkv;
    const int si = items[2 * it], ct = items[2 * it + 1];
    const int off = seq[5 * si], T = seq[5 * si + 1], start = seq[5 * si + 2], slot = seq[5 * si + 3];
    const int P = seq[5 * si + 4];
    const size_t row0 = (size_t)off * Hkv * G * D;
    const size_t kvoff = (size_t)slot * slot_elems * (KV8 ? 1 : 2);
    const void* kc = static_cast<const char*>(kcache) + kvoff;
    const void* vc = static_cast<const char*>(vcache) + kvoff;
    prefill_attn_block<D, NSUB, NWAVE, KV8>(q + row0, kc, vc, P > 0 ? pk : kc, P > 0 ? pv : vc, out + row0, nullptr,
                                            nullptr, T, start, P, Hkv, G, ldk, kh, 0, ct, 1, sl2, nullptr, 1L, 1L);
}

// split-K merge: out[row, :] = sum_s O_s exp2(m_s - M) / sum_s l_s exp2(m_s - M),
// M = max_s m_s (log2 domain).  One thread per 4 outputs.
template <int D>
__global__ __launch_bounds__(kBlock) void prefill_combine_kernel(const float* __restrict__ part_o,
                                                                const float* __restrict__ part_ml,
                                                                uint16_t* __restrict__ out, int rows, int nsplit) {
    const size_t idx = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= (size_t)rows * (D / 4)) return;
    const size_t row = idx / (D / 4);
    const int d = (int)(idx - row * (D / 4)) * 4;
    float M = -1e30f;
    for (int s = 0; s < nsplit; ++s) M = fmaxf(M, part_ml[((size_t)s * rows + row) * 2]);
    float L = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int s = 0; s < nsplit; ++s) {
        const size_t pr = (size_t)s * rows + row;
        const float2 ml = *reinterpret_cast<const float2*>(part_ml + pr * 2);
        const float w = __builtin_amdgcn_exp2f(ml.x - M);
        const float4 v = *reinterpret_cast<const float4*>(part_o + pr * D + d);
        L += ml.y * w;
        a0 += v.x * w;
        a1 += v.y * w;
        a2 += v.z * w;
        a3 += v.w * w;
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    const float f[4] = {a0 * inv, a1 * inv, a2 * inv, a3 * inv};
    *reinterpret_cast<uint2*>(out + row * D + d) = pack4(f);
}

template <int D, int NSUB, int NWAVE, bool KV8>
hipError_t launch_prefill(const uint16_t* q, const void* k, const void* v, const void* pk, const void* pv,
                          uint16_t* out, float* po, float* pml, int T, int start, int P, int Hkv, int G, int ldk,
                          int nsplit, float sl2, hipStream_t st) {
    constexpr int COLS = 32 * NSUB * NWAVE;
    const int ctiles = (T * G + COLS - 1) / COLS;
    prefill_attn_kernel<D, NSUB, NWAVE, KV8><<<dim3((unsigned)(ctiles * Hkv * nsplit)), NWAVE * kWave, 0, st>>>(
        q, k, v, pk, pv, out, po, pml, T, start, P, Hkv, G, ldk, ctiles, nsplit, sl2, nullptr, 1L,
        (long)T * G * Hkv);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || nsplit == 1) return e;
    const int rows = T * G * Hkv;
    const size_t n = (size_t)rows * (D / 4);
    prefill_combine_kernel<D><<<dim3((unsigned)((n + kBlock - 1) / kBlock)), kBlock, 0, st>>>(po, pml, out, rows,
                                                                                             nsplit);
    return hipGetLastError();
}

}  // namespace

// The decode step's shared-prefix attention on this kernel (called by
// dmcp_decode_attention, dmcp_kernels.hip): q [B, Hq, D] (one query token per
// row), prefix keys [0, *plen) of pk/pv ([Hkv, ldk, D]), partials written at
// index row * splits_total + split (split < nsplit) of the decode workspace.
// The grid is sized for the slot capacity; splits past *plen write empty
// partials (m = -1e30, l = 0).
hipError_t dmcp_launch_prefix_partials(const uint16_t* q, const void* pk, const void* pv, const int32_t* plen,
                                       float* part_o, float* part_ml, int B, int Hkv, int G, int D, int ldk,
                                       int nsplit, int splits_total, float sl2, int kv8, hipStream_t st) {
    constexpr int COLS = 32 * 4;  // variant 0: 4 waves x one 32-column unit
    const int ctiles = (B * G + COLS - 1) / COLS;
    const dim3 grid((unsigned)(ctiles * Hkv * nsplit));
#define DMCP_PFX(DD, K8)                                                                                          \
    prefill_attn_kernel<DD, 1, 4, K8><<<grid, 4 * kWave, 0, st>>>(q, pk, pv, pk, pv, nullptr, part_o, part_ml, B,    \
                                                                 ldk, 0, Hkv, G, ldk, ctiles, nsplit, sl2, plen,   \
                                                                 (long)splits_total, 1L)
    if (D == 64 && kv8) DMCP_PFX(64, true);
    else if (D == 64) DMCP_PFX(64, false);
    else if (D == 128 && kv8) DMCP_PFX(128, true);
    else if (D == 128) DMCP_PFX(128, false);
    else return hipErrorInvalidValue;
#undef DMCP_PFX
    return hipGetLastError();
}

extern "C" {

// q [T, Hq, D] (token-major, the rope_kv output); k/v: the sequence's slot
// [Hkv, ldk, D]; pk/pv: the shared-prefix slot (same layout) holding keys
// [0, P) -- P == 0 reads every key from k/v; out [T, Hq, D].  Query t sits at
// position start + t and sees keys [0, start + t].
// variant: waves per block, 0 = 4 (default), 1 = 8 (one 32-column unit per
// wave; two units per wave measured 3x slower at D = 64: 268 VGPRs, one wave
// per SIMD -- profiles/prefill_attn_r2.md).
// nsplit > 1 splits each tile's keys over that many blocks: part_o
// [nsplit, T*Hq, D] / part_ml [nsplit, T*Hq, 2] fp32 scratch, merged in a
// second kernel.
int dmcp_prefill_attention(const void* q, const void* k, const void* v, const void* pk, const void* pv, void* out,
                           void* part_o, void* part_ml, int T, int start, int P, int Hq, int Hkv, int D, int ldk,
                           float scale, int variant, int nsplit, int kv8, void* stream) {
    if (T <= 0) return 0;
    if (!q || !k || !v || !out || Hkv <= 0 || Hq % Hkv != 0 || start < 0 || P < 0 || P > start ||
        start + T > ldk || (P > 0 && (!pk || !pv)) || nsplit < 1 || nsplit > 64 ||
        (nsplit > 1 && (!part_o || !part_ml)))
        return hipErrorInvalidValue;
    if ((long)T * Hq > (1L << 28)) return hipErrorInvalidValue;
    const int G = Hq / Hkv;
    const float sl2 = scale * 1.4426950408889634f;
    auto st = (hipStream_t)stream;
    auto qq = (const uint16_t*)q;
    const void* ppk = P > 0 ? pk : k;
    const void* ppv = P > 0 ? pv : v;
    auto oo = (uint16_t*)out;
    auto po = (float*)part_o;
    auto pml = (float*)part_ml;
#define DMCP_PF(DD, NS, NW)                                                                                   \
    (kv8 ? launch_prefill<DD, NS, NW, true>(qq, k, v, ppk, ppv, oo, po, pml, T, start, P, Hkv, G, ldk, nsplit, sl2, \
                                            st)                                                                 \
         : launch_prefill<DD, NS, NW, false>(qq, k, v, ppk, ppv, oo, po, pml, T, start, P, Hkv, G, ldk, nsplit,   \
                                             sl2, st))
    if (D == 64) {
        switch (variant) {
            case 0: return DMCP_PF(64, 1, 4);
            case 1: return DMCP_PF(64, 1, 8);
            default: return hipErrorInvalidValue;
        }
    }
    if (D == 128) {
        switch (variant) {
            case 0: return DMCP_PF(128, 1, 4);
            case 1: return DMCP_PF(128, 1, 8);
            default: return hipErrorInvalidValue;
        }
    }
#undef DMCP_PF
    return hipErrorInvalidValue;
}

// Packed multi-sequence prefill attention.  q / out [Ttot, Hq, D]; caches
// [S, Hkv, ldk, D]; pk / pv: the shared-prefix slot ([Hkv, ldk, D]) for
// sequences whose prefix length is > 0.  items [nitems, 2] = (sequence, column
// tile) and seq [nseq, 5] = (token offset, T, start, slot, prefix length),
// int32 on the device; 4 waves x 32 columns per tile.
int dmcp_prefill_varlen(const void* q, const void* kc, const void* vc, const void* pk, const void* pv, void* out,
                        const void* items, const void* seq, int nitems, int Hq, int Hkv, int D, int ldk,
                        long slot_elems, float scale, int kv8, void* stream) {
    if (nitems <= 0) return 0;
    if (!q || !kc || !vc || !out || !items || !seq || Hkv <= 0 || Hq % Hkv != 0 || (long)nitems * Hkv > (1L << 31))
        return hipErrorInvalidValue;
    const int G = Hq / Hkv;
    const float sl2 = scale * 1.4426950408889634f;
    const dim3 grid((unsigned)(nitems * Hkv));
    auto st = (hipStream_t)stream;
    auto it = (const int32_t*)items;
    auto sq = (const int32_t*)seq;
#define DMCP_PV(DD, K8)                                                                                         \
    prefill_varlen_kernel<DD, 1, 4, K8><<<grid, 4 * kWave, 0, st>>>((const uint16_t*)q, kc, vc, pk, pv,           \
                                                                    (uint16_t*)out, it, sq, Hkv, G, ldk,          \
                                                                    (size_t)slot_elems, sl2)
    if (D == 64 && kv8) DMCP_PV(64, true);
    else if (D == 64) DMCP_PV(64, false);
    else if (D == 128 && kv8) DMCP_PV(128, true);
    else if (D == 128) DMCP_PV(128, false);
    else return hipErrorInvalidValue;
#undef DMCP_PV
    return hipGetLastError();
}

}  // extern "C"
