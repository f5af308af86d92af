// Fused decode GEMMs for gfx950 (MI355X, CDNA4): the four weight products of
// a decoder layer at decode-step row counts (M <= 128), each with the
// element-wise work around it folded into its prologue / epilogue, so a
// layer is QKV -> attention -> O -> gate/up -> down with no separate
// RMSNorm, RoPE/KV-append or SwiGLU launches:
//
//   EPI_ROPE_KV  rows  = RMSNorm(x) . Wqkv^T      -> RoPE(q), RoPE(k) + append k/v to the KV cache
//   EPI_SWIGLU   act   = silu(RMSNorm(x) . Wg^T) * (RMSNorm(x) . Wu^T)
//   EPI_RESID    resid += x . W^T                 (O and down projections)
//   EPI_BF16     out   = RMSNorm(x) . W^T         (LM head)
//
// RMSNorm's weight is folded into the following weight matrix on the host
// (W'[n, k] = W[n, k] * g[k], dmcp/models/llm.py), so the norm is a per-row
// scale rsqrt(mean(x^2) + eps) applied to the fp32 accumulator; the row sums
// of squares come from the same X fragments the MFMAs consume
// (v_dot2_f32_bf16, no extra loads).
//
// Shape of the work (decode: M rows << N, K): weight-streaming, HBM-bound.
// One block per 16-row weight block (or pair of blocks that the epilogue
// needs together: a RoPE pair d / d + D/2 of one head, a gate / up pair),
// its WK waves split K into contiguous ranges, every wave streams its W
// rows once with 16-B loads straight to VGPRs (A operand of
// v_mfma_f32_16x16x32_bf16; no LDS round trip, 'GEMV / M <= 16' row of the
// guide) and reads X (L2-resident, shared by every block) as the B operand,
// with a rolling register pipeline of 3-4 k-steps of loads in flight.  The WK partial tiles are summed
// through LDS in log2(WK) rounds and wave 0 runs the epilogue in the MFMA
// accumulator layout: lane (l16 = lane & 15, g = lane >> 4) holds output
// columns row0 + 4g + i (i < 4) of row m = 16 mt + l16, so every store is
// 4 consecutive bf16 (8 B) and a RoPE pair (d, d + D/2) is in one lane.
#include "dmcp_common.hpp"

namespace {

enum : int { EPI_ROPE_KV = 0, EPI_SWIGLU = 1, EPI_RESID = 2, EPI_BF16 = 3 };

struct FusedGemmArgs {
    const uint16_t* x;  // [M, K] bf16
    const uint16_t* w;  // [N, K] bf16
    uint16_t* out;      // SWIGLU: [M, inter]; RESID: residual [M, N] (read-modify-write); BF16: [M, N]
    int M, K, N;
    float eps;
    int inter;  // SWIGLU: intermediate size I (rows [0, I) gate, [I, 2I) up)
    // EPI_ROPE_KV
    const int32_t* pos;
    const int32_t* slot;
    const float2* cos_sin;  // [max_pos, D/2] (cos, sin)
    uint16_t* q_out;        // [M, Hq, D]
    void* k_cache;          // [S, Hkv, max_seq, D], bf16 or (kv8) fp8 e4m3
    void* v_cache;
    int Hq, Hkv, D, max_seq, max_pos, num_slots;
    int kv8;
};

template <int EPI>
struct EpiTraits {
    static constexpr int NB = (EPI == EPI_ROPE_KV || EPI == EPI_SWIGLU) ? 2 : 1;  // 16-row weight blocks per tile
    static constexpr bool NORM = EPI != EPI_RESID;
};

// first weight row of 16-row block nb of tile t
template <int EPI>
__device__ __forceinline__ int tile_row(const FusedGemmArgs& a, int t, int nb) {
    if constexpr (EPI == EPI_ROPE_KV) {
        const int pairs = a.D / 32;  // (d, d + D/2) block pairs per head
        const int hh = t / pairs, j = t - hh * pairs;
        return hh * a.D + 16 * j + nb * (a.D / 2);
    } else if constexpr (EPI == EPI_SWIGLU) {
        return 16 * t + nb * a.inter;
    } else {
        return 16 * t;
    }
}

// sum of squares of the 8 bf16 of a fragment, accumulated into acc
__device__ __forceinline__ float sumsq8(const uint4& v, float acc) {
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bf16x2_t p = __builtin_bit_cast(bf16x2_t, u[i]);
        acc = __builtin_amdgcn_fdot2_f32_bf16(p, p, acc, false);
    }
    return acc;
}

template <int MT, int WK, int EPI>
__global__ __launch_bounds__(WK * kWave) void fused_gemm_kernel(FusedGemmArgs a) {
    constexpr int NB = EpiTraits<EPI>::NB;
    constexpr bool NORM = EpiTraits<EPI>::NORM;
    constexpr int E = NB * MT * 4 + (NORM ? MT : 0);  // fp32 values per lane to reduce
    static_assert((WK & (WK - 1)) == 0 && WK >= 1 && WK <= 16, "WK must be a power of two <= 16");
    __shared__ float red[(WK > 1 ? WK / 2 : 1) * E * kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wk = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int l16 = lane & 15, g = lane >> 4;
    const int t = blockIdx.x;
    const int K = a.K;
    const int ksteps = K / 32;
    const int per = (ksteps + WK - 1) / WK;
    const int s0 = min(ksteps, wk * per), s1 = min(ksteps, s0 + per);
    const uint16_t* wp[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) wp[nb] = a.w + (size_t)(tile_row<EPI>(a, t, nb) + l16) * K + 8 * g;
    const uint16_t* xp[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) xp[mt] = a.x + (size_t)min(16 * mt + l16, a.M - 1) * K + 8 * g;
    f32x4_t acc[NB][MT];
    float ss[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        ss[mt] = 0.f;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[nb][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    // Rolling register pipeline: P k-steps of W and X loads in flight per
    // lane.  Slot j of the ring is consumed by the MFMAs of step s + j and at
    // once refilled with step s + j + P, so the wave never waits a full
    // memory round trip per k-step (a 2-deep load/compute loop was
    // latency-bound at 0.4-1.6 TB/s -- profiles/decode_step_r2_fused_v1*).
    // Loads in the steady-state loop are unconditional: a load under a
    // branch makes the compiler's wait-count pass fall back to vmcnt(0),
    // which serialises the pipeline again.
    constexpr int P = MT <= 6 ? 4 : 3;
    auto load_step = [&](uint4 (&wv)[NB], uint4 (&xv)[MT], int st) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) wv[nb] = *reinterpret_cast<const uint4*>(wp[nb] + 32 * st);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xv[mt] = *reinterpret_cast<const uint4*>(xp[mt] + 32 * st);
    };
    auto mma_step = [&](const uint4 (&wv)[NB], const uint4 (&xv)[MT]) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            if constexpr (NORM) ss[mt] = sumsq8(xv[mt], ss[mt]);
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
                acc[nb][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wv[nb]), as_bf16x8(xv[mt]),
                                                                     acc[nb][mt], 0, 0, 0);
        }
    };
    int s = s0;
    if (s1 - s0 >= P) {
        uint4 wf[P][NB], xf[P][MT];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            load_step(wf[j], xf[j], s0 + j);
            __builtin_amdgcn_sched_barrier(0);  // issue order = slot order (the loop's wait counts assume it)
        }
        for (; s + 2 * P <= s1; s += P) {
#pragma unroll
            for (int j = 0; j < P; ++j) {
                mma_step(wf[j], xf[j]);
                load_step(wf[j], xf[j], s + j + P);
                // keep the refill right behind its slot's MFMAs (the
                // scheduler otherwise sinks all refills below the next slots'
                // MFMAs, halving the loads in flight)
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int j = 0; j < P; ++j) mma_step(wf[j], xf[j]);  // drain
        s += P;
    }
    for (; s < s1; ++s) {  // remainder (< P steps)
        uint4 wv[NB], xv[MT];
        load_step(wv, xv, s);
        mma_step(wv, xv);
    }
    // K-split reduction across the block's waves: log2(WK) LDS rounds
#pragma unroll
    for (int half = WK / 2; half >= 1; half >>= 1) {
        __syncthreads();
        if (wk >= half && wk < 2 * half) {
            float* dst = red + (size_t)(wk - half) * E * kWave + lane;
            int e = 0;
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) dst[(e++) * kWave] = acc[nb][mt][i];
            if constexpr (NORM)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) dst[(e++) * kWave] = ss[mt];
        }
        __syncthreads();
        if (wk < half) {
            const float* src = red + (size_t)wk * E * kWave + lane;
            int e = 0;
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[nb][mt][i] += src[(e++) * kWave];
            if constexpr (NORM)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) ss[mt] += src[(e++) * kWave];
        }
    }
    if (wk != 0) return;
    // ---------------------------------------------------------------- epilogue
    const int r0 = tile_row<EPI>(a, t, 0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        float inv = 1.f;
        if constexpr (NORM) {
            float sq = ss[mt];
            sq += __shfl_xor(sq, 16, kWave);
            sq += __shfl_xor(sq, 32, kWave);
            inv = rsqrtf(sq / (float)K + a.eps);
        }
        const int m = 16 * mt + l16;
        if (m >= a.M) continue;
        float v[NB][4];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int i = 0; i < 4; ++i) v[nb][i] = acc[nb][mt][i] * inv;
        if constexpr (EPI == EPI_BF16) {
            *reinterpret_cast<uint2*>(a.out + (size_t)m * a.N + r0 + 4 * g) = pack4(v[0]);
        } else if constexpr (EPI == EPI_RESID) {
            uint2* rp = reinterpret_cast<uint2*>(a.out + (size_t)m * a.N + r0 + 4 * g);
            float r[4];
            unpack4(*rp, r);
#pragma unroll
            for (int i = 0; i < 4; ++i) r[i] += v[0][i];
            *rp = pack4(r);
        } else if constexpr (EPI == EPI_SWIGLU) {
            float o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = v[0][i] / (1.f + __expf(-v[0][i])) * v[1][i];
            *reinterpret_cast<uint2*>(a.out + (size_t)m * a.inter + r0 + 4 * g) = pack4(o);
        } else {  // EPI_ROPE_KV
            const int D = a.D, half = D / 2;
            const int hh = r0 / D;
            const int d0 = r0 - hh * D + 4 * g;  // < D/2: this lane's 4 dims and their partners d0 + D/2
            const int p = a.pos[m];
            float o1[4], o2[4];
            if (hh < a.Hq + a.Hkv) {  // q and k heads: rotate-half RoPE
                const float2* cs = a.cos_sin + (size_t)min(max(p, 0), a.max_pos - 1) * half + d0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float2 c = cs[i];
                    o1[i] = v[0][i] * c.x - v[1][i] * c.y;
                    o2[i] = v[1][i] * c.x + v[0][i] * c.y;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    o1[i] = v[0][i];
                    o2[i] = v[1][i];
                }
            }
            if (hh < a.Hq) {
                uint16_t* dst = a.q_out + ((size_t)m * a.Hq + hh) * D;
                *reinterpret_cast<uint2*>(dst + d0) = pack4(o1);
                *reinterpret_cast<uint2*>(dst + d0 + half) = pack4(o2);
                continue;
            }
            const int sl = a.slot[m];
            if (p < 0 || p >= a.max_seq || sl < 0 || sl >= a.num_slots) continue;  // padding row
            const int kv = hh < a.Hq + a.Hkv ? hh - a.Hq : hh - a.Hq - a.Hkv;
            void* cache = hh < a.Hq + a.Hkv ? a.k_cache : a.v_cache;
            const size_t off = (((size_t)sl * a.Hkv + kv) * a.max_seq + p) * D;
            if (a.kv8) {
                uint8_t* dst = static_cast<uint8_t*>(cache) + off;
                *reinterpret_cast<uint32_t*>(dst + d0) = pack_fp8x4_bf16r(o1);
                *reinterpret_cast<uint32_t*>(dst + d0 + half) = pack_fp8x4_bf16r(o2);
            } else {
                uint16_t* dst = static_cast<uint16_t*>(cache) + off;
                *reinterpret_cast<uint2*>(dst + d0) = pack4(o1);
                *reinterpret_cast<uint2*>(dst + d0 + half) = pack4(o2);
            }
        }
    }
}

template <int MT, int WK, int EPI>
hipError_t launch_mt(const FusedGemmArgs& a, int tiles, hipStream_t st) {
    fused_gemm_kernel<MT, WK, EPI><<<tiles, WK * kWave, 0, st>>>(a);
    return hipGetLastError();
}

// 16-wave blocks (<= 128 VGPRs per lane) only hold the pipeline of 2 row
// tiles; with more rows the block is capped at 8 waves (<= 256 VGPRs).
template <int WK, int EPI>
hipError_t launch_fused(const FusedGemmArgs& a, int tiles, hipStream_t st) {
    constexpr int W8 = WK > 8 ? 8 : WK;
    if (a.M <= 32) return launch_mt<2, WK, EPI>(a, tiles, st);
    if (a.M <= 64) return launch_mt<4, W8, EPI>(a, tiles, st);
    if (a.M <= 96) return launch_mt<6, W8, EPI>(a, tiles, st);
    if (a.M <= 128) return launch_mt<8, W8, EPI>(a, tiles, st);
    return hipErrorInvalidValue;
}

}  // namespace

extern "C" {

// Largest row count the fused GEMMs take (larger steps use hipBLASLt).
int dmcp_fused_gemm_max_rows() { return 128; }

// epi: 0 = ROPE_KV, 1 = SWIGLU, 2 = RESID, 3 = BF16 (see fused_gemm.hip).
// wk: waves per block splitting K (1, 2, 4, 8 or 16).  Shapes are validated
// by the host wrapper (dmcp/ops/hip.py::fused_gemm); the checks here only
// guard the tiling assumptions.
int dmcp_fused_gemm(int epi, int wk, const void* x, const void* w, void* out, int M, int K, int N, float eps,
                    int inter, const void* pos, const void* slot, const void* cos_sin, void* q_out, void* k_cache,
                    void* v_cache, int Hq, int Hkv, int D, int max_seq, int max_pos, int num_slots, int kv8,
                    void* stream) {
    if (M <= 0) return 0;
    if (M > 128 || K <= 0 || K % 32 != 0 || N <= 0 || !x || !w) return hipErrorInvalidValue;
    FusedGemmArgs a{(const uint16_t*)x, (const uint16_t*)w, (uint16_t*)out, M, K, N, eps, inter,
                    (const int32_t*)pos, (const int32_t*)slot, (const float2*)cos_sin, (uint16_t*)q_out,
                    k_cache, v_cache, Hq, Hkv, D, max_seq, max_pos, num_slots, kv8};
    auto st = (hipStream_t)stream;
    int tiles;
    switch (epi) {
        case EPI_ROPE_KV:
            if (D % 32 != 0 || D > 256 || N != (Hq + 2 * Hkv) * D || !pos || !slot || !cos_sin || !q_out ||
                !k_cache || !v_cache || max_pos <= 0)
                return hipErrorInvalidValue;
            tiles = N / 32;
            break;
        case EPI_SWIGLU:
            if (inter <= 0 || inter % 16 != 0 || N != 2 * inter || !out) return hipErrorInvalidValue;
            tiles = inter / 16;
            break;
        case EPI_RESID:
        case EPI_BF16:
            if (N % 16 != 0 || !out) return hipErrorInvalidValue;
            tiles = N / 16;
            break;
        default:
            return hipErrorInvalidValue;
    }
#define DMCP_FUSED_EPI(E)                                    \
    switch (wk) {                                            \
        case 4: return launch_fused<4, E>(a, tiles, st);    \
        case 8: return launch_fused<8, E>(a, tiles, st);    \
        case 16: return launch_fused<16, E>(a, tiles, st);  \
        default: return hipErrorInvalidValue;                \
    }
    switch (epi) {
        case EPI_ROPE_KV: DMCP_FUSED_EPI(EPI_ROPE_KV)
        case EPI_SWIGLU: DMCP_FUSED_EPI(EPI_SWIGLU)
        case EPI_RESID: DMCP_FUSED_EPI(EPI_RESID)
        default: DMCP_FUSED_EPI(EPI_BF16)
    }
#undef DMCP_FUSED_EPI
}

}  // extern "C"
