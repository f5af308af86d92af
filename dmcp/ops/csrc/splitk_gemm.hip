// Split-K decode GEMM with the residual add + RMSNorm of the next op folded
// into its reduction, for gfx950 (MI355X, CDNA4) -- the O and down
// projections of a decode step at 33-128 rows:
//
//   resid += bf16(x . W^T);   out = RMSNorm(resid) * g
//
// which the hipBLASLt path runs as F.linear + add_rmsnorm (two launches, the
// GEMM output written and re-read).  Shape of the work: M <= 128 rows, N x K
// weights streamed once from HBM; at N = 2048 a whole-K tiling gives 32-128
// blocks for 256 CUs (hipBLASLt: 0.7-1.6 TB/s on these shapes,
// profiles/gemm_blas_backends_r2.jsonl).  Here:
//
//   splitk_gemm_kernel   grid (N/64) x S: block (tile, s) computes the 64
//                        output columns n0..n0+63 over K slice s for every
//                        row, 4 waves x 16 weight rows (A operand of
//                        v_mfma_f32_16x16x32_bf16, 16-B loads straight to
//                        VGPRs), X fragments (L2-resident, shared by every
//                        block) as the B operand, a rolling register ring of
//                        P k-steps in flight; fp32 partial slab part[s][m][n].
//   splitk_reduce_norm   one block per row: sum of the S slabs, bf16 round
//                        (what F.linear returns), + residual (bf16 stream,
//                        written back), RMSNorm with weight g -> out.
//
// The reduction is a second launch, not an in-launch last-arriver combine:
// it needs the whole row for the norm anyway (cdna_hip_programming.md §5:
// combine in the next kernel when that kernel exists).
#include "dmcp_common.hpp"

namespace {

constexpr int kTileN = 64;  // output columns per block (4 waves x 16)

template <int MT>
__global__ __launch_bounds__(kBlock) void splitk_gemm_kernel(const uint16_t* __restrict__ x,
                                                             const uint16_t* __restrict__ w,
                                                             float* __restrict__ part, int M, int K, int N,
                                                             int ks) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int l16 = lane & 15, g = lane >> 4;
    const int n0 = blockIdx.x * kTileN + 16 * wv;
    const int s = blockIdx.y;
    const int k0 = s * ks;
    const int steps = ks / 32;
    const uint16_t* wp = w + (size_t)(n0 + l16) * K + k0 + 8 * g;
    const uint16_t* xp[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) xp[mt] = x + (size_t)min(16 * mt + l16, M - 1) * K + k0 + 8 * g;
    f32x4_t acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    constexpr int P = MT <= 4 ? 6 : 4;  // k-steps of loads in flight per lane
    auto load_step = [&](uint4& wf, uint4 (&xf)[MT], int st) {
        wf = *reinterpret_cast<const uint4*>(wp + 32 * st);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xf[mt] = *reinterpret_cast<const uint4*>(xp[mt] + 32 * st);
    };
    auto mma_step = [&](const uint4& wf, const uint4 (&xf)[MT]) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wf), as_bf16x8(xf[mt]), acc[mt], 0, 0, 0);
    };
    int st = 0;
    if (steps >= P) {
        uint4 wr[P], xr[P][MT];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            load_step(wr[j], xr[j], j);
            __builtin_amdgcn_sched_barrier(0);
        }
        for (; st + 2 * P <= steps; st += P) {
#pragma unroll
            for (int j = 0; j < P; ++j) {
                mma_step(wr[j], xr[j]);
                load_step(wr[j], xr[j], st + j + P);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int j = 0; j < P; ++j) mma_step(wr[j], xr[j]);
        st += P;
    }
    for (; st < steps; ++st) {
        uint4 wf, xf[MT];
        load_step(wf, xf, st);
        mma_step(wf, xf);
    }
    // accumulator layout: lane (l16, g) holds columns n0 + 4g + i of row 16 mt + l16
    float* dst = part + (size_t)s * M * N + n0 + 4 * g;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + l16;
        if (m < M) *reinterpret_cast<float4*>(dst + (size_t)m * N) = make_float4(acc[mt][0], acc[mt][1], acc[mt][2], acc[mt][3]);
    }
}

// Variant 1: the X slice goes through LDS once per block (the register-direct
// kernel above re-reads every X fragment in each of the 4 waves: 1.3-1.8x
// slower than hipBLASLt, profiles/splitk_gemm_r2_v1.jsonl).  64-deep chunks of
// all MP = 16 MT rows, two buffers, one barrier per chunk; 16-B pieces
// XOR-swizzled by row (piece ^ (row & 7)) so a wave's ds_read_b128 of 16 rows
// x 4 pieces is at most 2-way conflicted.  W stays register-direct with a
// ring of 4 k-steps.  Needs the K slice to be a multiple of 128.
// SWI: x is the gate/up GEMM output [M, 2K] and the operand is
// silu(gate) * up, computed while the slice is staged into LDS (the SwiGLU
// kernel's fp32 math and bf16 rounding), so the down projection reads the
// gate/up rows directly and no SwiGLU launch or activation buffer exists.
__device__ __forceinline__ uint4 swiglu8(const uint4& gv, const uint4& uv) {
    float gf[8], uf[8], o[8];
    unpack8(gv, gf);
    unpack8(uv, uf);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = gf[j] / (1.f + __expf(-gf[j])) * uf[j];
    return pack8(o);
}

template <int MT, bool SWI = false>
__global__ __launch_bounds__(kBlock) void splitk_gemm_lds_kernel(const uint16_t* __restrict__ x,
                                                                 const uint16_t* __restrict__ w,
                                                                 float* __restrict__ part, int M, int K, int N,
                                                                 int ks) {
    constexpr int MP = 16 * MT;
    constexpr int NP = MP * 8 / kBlock;  // 16-B X pieces per thread per chunk
    static_assert(NP >= 1 && MP * 8 % kBlock == 0, "MT must be even");
    __shared__ uint4 xs[2][MP * 8];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    const int l16 = lane & 15, g = lane >> 4;
    const int n0 = blockIdx.x * kTileN + 16 * wv;
    const int s = blockIdx.y;
    const int k0 = s * ks;
    const int steps = ks / 32, chunks = ks / 64;
    const uint16_t* wp = w + (size_t)(n0 + l16) * K + k0 + 8 * g;
    // this thread's X pieces: row pr[i], piece pc[i] of every chunk
    const uint16_t* xp[NP];
    int so[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int p = tid + i * kBlock;
        const int row = p >> 3, pc = p & 7;
        xp[i] = x + (size_t)min(row, M - 1) * (SWI ? 2 * K : K) + k0 + 8 * pc;
        so[i] = row * 8 + (pc ^ (row & 7));
    }
    f32x4_t acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    uint4 wr[4], xg[NP], xu[SWI ? NP : 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) wr[j] = *reinterpret_cast<const uint4*>(wp + 32 * min(j, steps - 1));
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const uint4 a = *reinterpret_cast<const uint4*>(xp[i]);
        if constexpr (SWI) xs[0][so[i]] = swiglu8(a, *reinterpret_cast<const uint4*>(xp[i] + K));
        else xs[0][so[i]] = a;
    }
    __syncthreads();
    for (int c = 0; c < chunks; c += 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // chunk c + h in buffer h
            const int cn = min(c + h + 1, chunks - 1);
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                xg[i] = *reinterpret_cast<const uint4*>(xp[i] + 64 * cn);
                if constexpr (SWI) xu[i] = *reinterpret_cast<const uint4*>(xp[i] + K + 64 * cn);
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int j = 2 * h + kk;  // ring slot of step 2 (c + h) + kk
                uint4 xf[MT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const int row = 16 * mt + l16;
                    xf[mt] = xs[h][row * 8 + ((4 * kk + g) ^ (row & 7))];
                }
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wr[j]), as_bf16x8(xf[mt]), acc[mt],
                                                                      0, 0, 0);
                wr[j] = *reinterpret_cast<const uint4*>(wp + 32 * min(2 * (c + h) + kk + 4, steps - 1));
            }
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                if constexpr (SWI) xs[h ^ 1][so[i]] = swiglu8(xg[i], xu[i]);
                else xs[h ^ 1][so[i]] = xg[i];
            }
            __syncthreads();
        }
    }
    float* dst = part + (size_t)s * M * N + n0 + 4 * g;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + l16;
        if (m < M)
            *reinterpret_cast<float4*>(dst + (size_t)m * N) = make_float4(acc[mt][0], acc[mt][1], acc[mt][2], acc[mt][3]);
    }
}

template <int VPT>
__global__ __launch_bounds__(kBlock) void splitk_reduce_norm_kernel(const float* __restrict__ part, int S,
                                                                    uint16_t* __restrict__ resid,
                                                                    const uint16_t* __restrict__ gw,
                                                                    uint16_t* __restrict__ out, int M, int N,
                                                                    float eps) {
    const int m = blockIdx.x;
    const int nvec = N >> 3;
    float h[VPT][8];
    uint4 rv[VPT], wv[VPT];
    uint4* rr = reinterpret_cast<uint4*>(resid + (size_t)m * N);
    const uint4* wr = reinterpret_cast<const uint4*>(gw);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            rv[i] = rr[idx];
            wv[i] = wr[idx];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) h[i][j] = 0.f;
    }
    for (int s = 0; s < S; ++s) {
        const float4* pp = reinterpret_cast<const float4*>(part + ((size_t)s * M + m) * N);
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            const int idx = threadIdx.x + i * kBlock;
            if (idx < nvec) {
                const float4 a = pp[2 * idx], b = pp[2 * idx + 1];
                h[i][0] += a.x; h[i][1] += a.y; h[i][2] += a.z; h[i][3] += a.w;
                h[i][4] += b.x; h[i][5] += b.y; h[i][6] += b.z; h[i][7] += b.w;
            }
        }
    }
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            float y[8], r[8];
            unpack8(pack8(h[i]), y);  // the GEMM output as F.linear rounds it
            unpack8(rv[i], r);
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] += r[j];
            const uint4 packed = pack8(y);
            rr[idx] = packed;
            unpack8(packed, h[i]);  // normalise the bf16-rounded stream (add_rmsnorm's order)
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
    for (int i = 0; i < kBlock / kWave; ++i) tot += red[i];
    const float inv = rsqrtf(tot / (float)N + eps);
    uint4* orow = reinterpret_cast<uint4*>(out + (size_t)m * N);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            float gv[8], o[8];
            unpack8(wv[i], gv);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = h[i][j] * inv * gv[j];
            orow[idx] = pack8(o);
        }
    }
}

// QKV variant of the reduction: the row's slabs summed and bf16-rounded
// into LDS (what F.linear returns), then rotate-half RoPE on q and k, q
// written out, k / v appended to the KV cache (bf16 or, KV8, fp8 e4m3) at
// (slot[t], :, pos[t], :) -- dmcp_kernels.hip::rope_kv_kernel over an LDS row.
template <bool KV8>
__global__ __launch_bounds__(kBlock) void splitk_reduce_rope_kernel(
    const float* __restrict__ part, int S, int M, const int32_t* __restrict__ pos, const int32_t* __restrict__ slot,
    const float2* __restrict__ cos_sin, uint16_t* __restrict__ q_out, void* __restrict__ k_cache,
    void* __restrict__ v_cache, int Hq, int Hkv, int D, int max_seq, int max_pos, int num_slots) {
    __shared__ uint4 rowbuf[8192 / 8];
    const int t = blockIdx.x;
    const int N = (Hq + 2 * Hkv) * D;
    const int nvec = N >> 3;
    for (int idx = threadIdx.x; idx < nvec; idx += kBlock) {
        float h[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < S; ++s) {
            const float4* pp = reinterpret_cast<const float4*>(part + ((size_t)s * M + t) * N);
            const float4 a = pp[2 * idx], b = pp[2 * idx + 1];
            h[0] += a.x; h[1] += a.y; h[2] += a.z; h[3] += a.w;
            h[4] += b.x; h[5] += b.y; h[6] += b.z; h[7] += b.w;
        }
        rowbuf[idx] = pack8(h);
    }
    __syncthreads();
    const uint16_t* row = reinterpret_cast<const uint16_t*>(rowbuf);
    const int p = pos[t];
    const int sl = slot[t];
    const bool write_cache = (p >= 0 && p < max_seq && sl >= 0 && sl < num_slots);
    const int half = D >> 1;
    const int quads = half >> 2;
    const float2* cs = cos_sin + (size_t)min(max(p, 0), max_pos - 1) * half;
    const int units = (Hq + Hkv) * quads;
    for (int u = threadIdx.x; u < units; u += kBlock) {
        const int hh = u / quads;
        const int d0 = (u - hh * quads) * 4;
        const uint16_t* src = row + (size_t)hh * D;
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
        const size_t kofs = (((size_t)sl * Hkv + (hh - Hq)) * max_seq + p) * D;
        if constexpr (KV8) {
            uint8_t* dst = static_cast<uint8_t*>(k_cache) + kofs;
            *reinterpret_cast<uint32_t*>(dst + d0) = pack_fp8x4(o1);
            *reinterpret_cast<uint32_t*>(dst + half + d0) = pack_fp8x4(o2);
        } else {
            uint16_t* dst = static_cast<uint16_t*>(k_cache) + kofs;
            *reinterpret_cast<uint2*>(dst + d0) = pack4(o1);
            *reinterpret_cast<uint2*>(dst + half + d0) = pack4(o2);
        }
    }
    if (!write_cache) return;
    const int vvec = (Hkv * D) >> 3;
    const uint4* vsrc = rowbuf + (((Hq + Hkv) * D) >> 3);
    for (int u = threadIdx.x; u < vvec; u += kBlock) {
        const int e = u << 3;
        const int kh = e / D;
        const int d = e - kh * D;
        const size_t vofs = (((size_t)sl * Hkv + kh) * max_seq + p) * D + d;
        if constexpr (KV8)
            *reinterpret_cast<uint2*>(static_cast<uint8_t*>(v_cache) + vofs) = bf16x8_to_fp8x8(vsrc[u]);
        else
            *reinterpret_cast<uint4*>(static_cast<uint16_t*>(v_cache) + vofs) = vsrc[u];
    }
}

template <int MT>
hipError_t launch_gemm(const uint16_t* x, const uint16_t* w, float* part, int M, int K, int N, int S, int variant,
                       hipStream_t st) {
    if (variant == 2)
        splitk_gemm_lds_kernel<MT, true><<<dim3(N / kTileN, S), kBlock, 0, st>>>(x, w, part, M, K, N, K / S);
    else if (variant == 1)
        splitk_gemm_lds_kernel<MT><<<dim3(N / kTileN, S), kBlock, 0, st>>>(x, w, part, M, K, N, K / S);
    else
        splitk_gemm_kernel<MT><<<dim3(N / kTileN, S), kBlock, 0, st>>>(x, w, part, M, K, N, K / S);
    return hipGetLastError();
}

}  // namespace

extern "C" {

// resid[M, N] += bf16(x[M, K] . w[N, K]^T); out = RMSNorm(resid) * g.
// part: fp32 workspace of S * M * N.  Shapes checked by the host wrapper
// (dmcp/ops/hip.py::linear_resid_norm); the checks here guard the tiling.
// variant 0: register-direct X; 1: X staged through LDS (K % (128 S) == 0);
// 2: as 1 with x = gate/up rows [M, 2K] and the operand silu(gate) * up.
int dmcp_splitk_resid_norm(const void* x, const void* w, void* part, void* resid, const void* g, void* out, int M,
                           int K, int N, int S, float eps, int variant, void* stream) {
    if (M <= 0) return 0;
    if (M > 128 || S <= 0 || N % kTileN != 0 || K % (32 * S) != 0 || N % 8 != 0 || N > 8 * 4 * kBlock || !x ||
        !w || !part || !resid || !g || !out || variant < 0 || variant > 2 || (variant >= 1 && K % (128 * S) != 0))
        return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    auto xx = (const uint16_t*)x;
    auto ww = (const uint16_t*)w;
    auto pp = (float*)part;
    hipError_t e;
    const int mt = (M + 15) / 16;
    if (mt <= 2) e = launch_gemm<2>(xx, ww, pp, M, K, N, S, variant, st);
    else if (mt <= 4) e = launch_gemm<4>(xx, ww, pp, M, K, N, S, variant, st);
    else if (mt <= 6) e = launch_gemm<6>(xx, ww, pp, M, K, N, S, variant, st);
    else e = launch_gemm<8>(xx, ww, pp, M, K, N, S, variant, st);
    if (e != hipSuccess) return e;
    const int vpt = (N / 8 + kBlock - 1) / kBlock;
    auto rr = (uint16_t*)resid;
    auto gg = (const uint16_t*)g;
    auto oo = (uint16_t*)out;
    if (vpt == 1) splitk_reduce_norm_kernel<1><<<M, kBlock, 0, st>>>(pp, S, rr, gg, oo, M, N, eps);
    else if (vpt == 2) splitk_reduce_norm_kernel<2><<<M, kBlock, 0, st>>>(pp, S, rr, gg, oo, M, N, eps);
    else splitk_reduce_norm_kernel<4><<<M, kBlock, 0, st>>>(pp, S, rr, gg, oo, M, N, eps);
    return hipGetLastError();
}

// q_out[M, Hq, D] = RoPE(q), k/v appended to the caches, of qkv = x . w^T
// (w [(Hq + 2 Hkv) D, K]); what F.linear + rope_kv compute.  part: fp32
// workspace of S * M * N.
int dmcp_splitk_rope_kv(const void* x, const void* w, void* part, const void* pos, const void* slot,
                        const void* cos_sin, void* q_out, void* k_cache, void* v_cache, int M, int K, int Hq, int Hkv,
                        int D, int max_seq, int max_pos, int num_slots, int kv8, int S, int variant, void* stream) {
    if (M <= 0) return 0;
    const int N = (Hq + 2 * Hkv) * D;
    if (M > 128 || S <= 0 || D % 16 != 0 || N % kTileN != 0 || N > 8192 || K % (32 * S) != 0 || !x || !w ||
        !part || !pos || !slot || !cos_sin || !q_out || !k_cache || !v_cache || max_pos <= 0 || variant < 0 ||
        variant > 1 || (variant == 1 && K % (128 * S) != 0))
        return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    auto xx = (const uint16_t*)x;
    auto ww = (const uint16_t*)w;
    auto pp = (float*)part;
    hipError_t e;
    const int mt = (M + 15) / 16;
    if (mt <= 2) e = launch_gemm<2>(xx, ww, pp, M, K, N, S, variant, st);
    else if (mt <= 4) e = launch_gemm<4>(xx, ww, pp, M, K, N, S, variant, st);
    else if (mt <= 6) e = launch_gemm<6>(xx, ww, pp, M, K, N, S, variant, st);
    else e = launch_gemm<8>(xx, ww, pp, M, K, N, S, variant, st);
    if (e != hipSuccess) return e;
    if (kv8)
        splitk_reduce_rope_kernel<true><<<M, kBlock, 0, st>>>(pp, S, M, (const int32_t*)pos, (const int32_t*)slot,
                                                              (const float2*)cos_sin, (uint16_t*)q_out, k_cache,
                                                              v_cache, Hq, Hkv, D, max_seq, max_pos, num_slots);
    else
        splitk_reduce_rope_kernel<false><<<M, kBlock, 0, st>>>(pp, S, M, (const int32_t*)pos, (const int32_t*)slot,
                                                               (const float2*)cos_sin, (uint16_t*)q_out, k_cache,
                                                               v_cache, Hq, Hkv, D, max_seq, max_pos, num_slots);
    return hipGetLastError();
}

}  // extern "C"
