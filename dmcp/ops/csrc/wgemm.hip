// Weight-streaming GEMM for the decode step (gfx950 / MI355X, CDNA4):
//
//   Y[M, N] = X[M, K] . W[N, K]^T      bf16 in, fp32 accumulate,  M <= 512
//
// At the enrichment operating point (256 sequences + jump-forward rows, ~300
// rows per step) every projection streams its whole weight matrix from HBM
// once per step while the activations are a few MB (L2-resident).
// hipBLASLt tiles M in 64-row blocks spread over all 8 XCDs, so each weight
// tile leaves HBM once per M tile: 0.6-2 TB/s of weight traffic at 320 rows
// (profiles/decode_step_320rows_fp8_r3_kernel_stats.csv: 91 us of GEMMs per
// layer against ~20 us at the HBM roofline).  Here:
//
//   * a block owns NB weight rows (64, or 128 = 64 gate + 64 up rows of the
//     same intermediate columns) and ALL rows of its M part: the weight tile
//     is read once and the M parts of one tile run on the SAME XCD (block
//     ids congruent mod 8, dispatched back to back), so the second part's
//     read is an L2 hit;
//   * both operands reach LDS by LDS-DMA (global_load_lds_dwordx4: full
//     128-B lines, no VGPR round trip) into a 3-stage ring of 64-deep K
//     chunks, two stages in flight while one is computed, one counted
//     vmcnt + raw barrier per chunk -- HBM latency needs ~60 KB in flight
//     per CU and a block's compute per chunk is a fraction of one latency;
//     with register-direct X loads every X wait also waited for the weight
//     loads issued before it (vmcnt retires in order): 2x slower than
//     hipBLASLt;
//   * LDS images are [rows][8 x 16 B] with chunk j of row r in slot
//     j ^ (r & 7) (the swizzle applied on the DMA's source address):
//     conflict-free ds_read_b128 of both MFMA operands;
//   * v_mfma_f32_16x16x32_bf16: A = 16 weight rows x 32 k, B = 32 k x 16 X
//     rows, C = Y^T tile (lane: 4 consecutive output columns of one row);
//   * the bound (profiles/wgemm_parts_r3.txt): each CU ingests its weight
//     tile at ~23 KB/us and its activation rows at ~42 KB/us through the
//     same load path, t ~= W_block / 23 + X_block / 42 (KB, us); 64 / 128
//     weight rows x the M part already minimise that for ~256 blocks;
//   * split-K (S > 1) writes fp32 partials, reduced by the fused consumers
//     below (residual + RMSNorm of the next op; RoPE + KV-cache append);
//     MODE_SWIGLU writes silu(gate) * up directly (no gate/up activation in
//     HBM, no SwiGLU launch);
//   * MODE_ARGMAX is the LM head + the grammar-masked greedy selection: each
//     block reduces its tile's vocabulary columns of every row to one
//     (max, id) pair under the row's mask bitset (the grammar state's mask
//     row), a tiny kernel reduces the pairs per row -- the [rows, vocab]
//     logits never exist (at 128,256 ids and 512 rows: 131 MB written and
//     read back per step by F.linear + masked_argmax).
#include "dmcp_common.hpp"

namespace {

constexpr int kKC = 64;  // K per LDS stage
constexpr int MODE_BF16 = 0, MODE_PART = 1, MODE_SWIGLU = 2, MODE_ARGMAX = 3;

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// LDS-DMA (global_load_lds_dwordx4): each lane's 16 source bytes land at
// the wave-uniform LDS base + 16 * lane, with no VGPR round trip; counted on
// vmcnt like any vector load.
// AUX: cache-policy bits of the load (2 = nt: streamed, evicted first from L2)
template <int AUX = 0>
__device__ __forceinline__ void glds16(const void* src, uint4* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds_base, 16, 0, AUX);
}

template <int NB, int MT, int MR, int MODE, int ST, int AUXW = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1))) void wgemm_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                       uint16_t* __restrict__ y, float* __restrict__ part, int M, int N,
                                                       int K, int ks, int S, int ntiles, int mparts, int mrows,
                                                       int I, const uint32_t* __restrict__ masks,
                                                       const int32_t* __restrict__ midx, int n_masks, int wwords) {
    constexpr int NF = NB / 16;         // A fragments (16 weight rows each)
    // X rows staged per block (a multiple of 32, <= 4 waves x MT 16-row
    // tiles): the M part rounded up to 32 rows, not to 64 -- at 320 rows
    // (two parts of 160) the X image is 160 rows instead of 192, and X is
    // most of the bytes each CU stages (profiles/decode_late_ab_r3.txt)
    static_assert(MR % 32 == 0 && MR <= MT * 64 && MR > (MT - 1) * 64, "MR: staged X rows");
    constexpr int WCH = NB * 8;         // 16-B chunks of a stage's weight image [NB][64 k]
    constexpr int SCH = WCH + MR * 8;   // ... plus the X image [MR][64 k]
    constexpr int WI = NB / 32;         // 1-KiB LDS-DMA pieces (8 rows x 128 B) per wave per stage: weights
    constexpr int XI = MR / 32;         //                                                          X rows
    constexpr int GL = WI + XI;         // LDS-DMA instructions per wave per stage
    // ONE shared array (a second __shared__ object can make hipcc wait vmcnt(0)
    // before every LDS read, draining the DMA ring: cdna_hip_programming.md §5)
    __shared__ uint4 lds[ST * SCH];

    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    const int l16 = lane & 15, g = lane >> 4;
    // block -> (weight tile nt, K slice s, M part mp); the M parts of one
    // (nt, s) unit share blockIdx % 8 (one XCD) and consecutive dispatch slots
    const int units = ntiles * S;
    int u, mp;
    if ((units & 7) == 0) {
        const int j = blockIdx.x >> 3;
        u = (j / mparts) * 8 + (blockIdx.x & 7);
        mp = j % mparts;
    } else {  // XCD-contiguous ranges (bijective for any grid): a unit's M parts on one XCD
        const int nblk = units * mparts, b = blockIdx.x;
        const int xcd = b & 7, q8 = nblk >> 3, r8 = nblk & 7;
        const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
        u = L / mparts;
        mp = L % mparts;
    }
    const int nt = u % ntiles, s = u / ntiles;
    const int k0 = s * ks;
    const int chunks = ks / kKC;
    const int m_lo = mp * mrows;
    const int m_hi = min(M, m_lo + mrows);
    const int mw = wv * (MT * 16);                 // this wave's first row inside the part
    int mtv = (m_hi - m_lo - mw + 15) / 16;        // valid 16-row tiles of this wave (wave-uniform)
    mtv = max(0, min(MT, mtv));

    // weight rows of this block: NB contiguous rows, or (SwiGLU) 64 gate rows
    // n0h.. and the 64 up rows I + n0h..
    const int n0 = nt * NB;
    const int n0h = nt * (NB / 2);
    auto wrow = [&](int r) -> int {
        if constexpr (MODE == MODE_SWIGLU) return r < NB / 2 ? n0h + r : I + n0h + (r - NB / 2);
        else return n0 + r;
    };
    // LDS images [rows][8 x 16 B], chunk j of row r stored at slot j ^ (r & 7)
    // (conflict-free ds_read_b128 of the fragments); LDS-DMA writes lane-linear,
    // so the swizzle goes on each lane's SOURCE address: lane L of a piece
    // fills row base + L / 8, slot L % 8 with logical chunk (L % 8) ^ (row & 7)
    const uint16_t* wsrc[WI];
    const uint16_t* xsrc[XI];
#pragma unroll
    for (int i = 0; i < WI; ++i) {
        const int r = (wv * WI + i) * 8 + (lane >> 3);
        wsrc[i] = w + (size_t)wrow(r) * K + k0 + (((lane & 7) ^ (r & 7)) * 8);
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {
        const int r = (wv * XI + i) * 8 + (lane >> 3);
        xsrc[i] = x + (size_t)min(m_lo + r, M - 1) * K + k0 + (((lane & 7) ^ (r & 7)) * 8);
    }
    auto issue = [&](int c, int slot) {
        uint4* base = lds + slot * SCH;
#pragma unroll
        for (int i = 0; i < WI; ++i) glds16<AUXW>(wsrc[i] + c * kKC, base + (wv * WI + i) * 64);
#pragma unroll
        for (int i = 0; i < XI; ++i) glds16(xsrc[i] + c * kKC, base + WCH + (wv * XI + i) * 64);
    };

    f32x4_t acc[NF][MT];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[f][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // Both 32-deep k steps' operand fragments are read from LDS before the
    // first MFMA of the chunk, the second step's reads overlapping the first
    // step's MFMAs: one exposed LDS latency per chunk instead of one per
    // fragment group.  At one wave per SIMD (the LDS ring holds one block per
    // CU) nothing else hides those latencies: the compiler's register-lean
    // schedule (2 A fragments live, lgkmcnt(0) before every 3-6 MFMAs) left
    // the matrix cores idle ~2/3 of the time (the 320-row gate/up GEMM with its
    // loads switched off: 32 -> 29 us, whole kernel 40 -> 38 us against
    // ~10 us of MFMA; the rest is the CU's load path: profiles/wgemm_parts_r3.txt).
    auto compute = [&](const uint4* st) {
        const uint4* wl = st;
        const uint4* xl = st + WCH;
        bf16x8_t b[2][MT], a[2][NF];
        auto load = [&](int kk) {
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                // rows past the staged image (the last wave's spare tile
                // when MR < MT * 64) read the image's last row; their
                // results are never stored (mtv / m_hi)
                const int r = min(mw + 16 * t + l16, MR - 1);
                b[kk][t] = as_bf16x8(xl[r * 8 + ((4 * kk + g) ^ (r & 7))]);
            }
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int r = 16 * f + l16;
                a[kk][f] = as_bf16x8(wl[r * 8 + ((4 * kk + g) ^ (r & 7))]);
            }
        };
        auto mma = [&](int kk) {
#pragma unroll
            for (int f = 0; f < NF; ++f)
                // every tile, valid or not: the waves meet at a barrier per
                // chunk, so a wave's idle tiles cost no wall time, and a
                // per-tile branch breaks back-to-back MFMA issue
#pragma unroll
                for (int t = 0; t < MT; ++t)
                    acc[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][f], b[kk][t], acc[f][t], 0, 0, 0);
        };
        // k step 0's reads, then its MFMAs with k step 1's reads threaded
        // between them (one read per RM MFMAs, pinned: the scheduler would
        // sink each read to its use), then k step 1's MFMAs.  At most
        // NF + MT <= 12 reads are in flight, within lgkmcnt's range, so the
        // waits stay counted (22 queued reads made the compiler wait for 0).
        constexpr int NR = NF + MT;            // fragment reads per k step
        constexpr int NM = NF * MT;            // MFMAs per k step
        constexpr int RM = NM / NR > 0 ? NM / NR : 1;
        load(0);
        __builtin_amdgcn_sched_barrier(0);
        load(1);
        mma(0);
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one DS read
            __builtin_amdgcn_sched_group_barrier(0x008, RM, 0);  // RM MFMAs
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);      // the rest
        __builtin_amdgcn_sched_barrier(0);
        mma(1);
    };

    // ST-stage ring, ST - 1 stages in flight: wait for this wave's pieces of
    // stage c (counted vmcnt, the next stage may stay in flight), one raw
    // barrier (every wave's pieces landed; every wave done reading the slot
    // about to be refilled), refill, compute.  No __syncthreads() in the loop:
    // its fence would drain the DMA ring (vmcnt(0)).
#pragma unroll
    for (int j = 0; j < ST - 1; ++j)
        if (j < chunks) issue(j, j);
    for (int c = 0; c < chunks; ++c) {
        if (c + ST - 2 < chunks) {
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(GL * (ST - 2)) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        }
        if (c + ST - 1 < chunks) issue(c + ST - 1, (c + ST - 1) % ST);
        compute(lds + (c % ST) * SCH);
    }

    // epilogue: lane (l16, g) holds Y[row m_lo + mw + 16t + l16][col 16f + 4g + i]
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        if (t >= mtv) continue;
        const int m = m_lo + mw + 16 * t + l16;
        if constexpr (MODE == MODE_ARGMAX) {
            // masked max of this row over the tile's NB columns: each lane its
            // 4 NF columns, then across the 4 lane groups g (every lane takes
            // part in the shuffles; rows past the part only skip the store).
            // Values are bf16-rounded (what F.linear + masked_argmax compare),
            // ties go to the lowest id.
            float bv = -INFINITY;
            int bi = 0x7fffffff;
            if (m < m_hi) {
                int mr = midx ? midx[m] : 0;
                mr = mr < 0 ? 0 : (mr >= n_masks ? n_masks - 1 : mr);
                const uint32_t* mrow = masks + (size_t)mr * wwords + (n0 >> 5);
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const uint32_t word = mrow[(16 * f + 4 * g) >> 5];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int c = 16 * f + 4 * g + i;
                        if ((word >> (c & 31)) & 1u) {
                            const float x = bf2f(f2bf(acc[f][t][i]));
                            if (x > bv) { bv = x; bi = n0 + c; }  // columns ascend: strict > keeps the lowest
                        }
                    }
                }
            }
#pragma unroll
            for (int msk = 16; msk < kWave; msk <<= 1) {
                const float ob = __shfl_xor(bv, msk, kWave);
                const int oi = __shfl_xor(bi, msk, kWave);
                if (ob > bv || (ob == bv && oi < bi)) { bv = ob; bi = oi; }
            }
            if (m < m_hi && g == 0)
                reinterpret_cast<float2*>(part)[(size_t)nt * M + m] = make_float2(bv, __int_as_float(bi));
            continue;
        }
        if (m >= m_hi) continue;
        if constexpr (MODE == MODE_SWIGLU) {
#pragma unroll
            for (int f = 0; f < NF / 2; ++f) {
                float o[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {  // gate / up rounded to bf16 as the unfused GEMM output is
                    const float gg = bf2f(f2bf(acc[f][t][i])), uu = bf2f(f2bf(acc[f + NF / 2][t][i]));
                    o[i] = silu_f(gg) * uu;
                }
                *reinterpret_cast<uint2*>(y + (size_t)m * I + n0h + 16 * f + 4 * g) = pack4(o);
            }
        } else if constexpr (MODE == MODE_PART) {
            float* dst = part + ((size_t)s * M + m) * N + n0 + 4 * g;
#pragma unroll
            for (int f = 0; f < NF; ++f)
                *reinterpret_cast<float4*>(dst + 16 * f) =
                    make_float4(acc[f][t][0], acc[f][t][1], acc[f][t][2], acc[f][t][3]);
        } else {
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const float o[4] = {acc[f][t][0], acc[f][t][1], acc[f][t][2], acc[f][t][3]};
                *reinterpret_cast<uint2*>(y + (size_t)m * N + n0 + 16 * f + 4 * g) = pack4(o);
            }
        }
    }
}

// split-K slices whose partials the reductions below load at once
constexpr int RSU = 4;

// split-K reduction + residual add + RMSNorm of the next op (one block per
// row): resid += bf16(sum_s part[s]); out = RMSNorm(resid) * gw.  The GEMM
// output is rounded to bf16 before the add and the stream after it (what
// F.linear + add_rmsnorm compute).
template <int VPT>
__global__ __launch_bounds__(kBlock) void reduce_resid_norm_kernel(const float* __restrict__ part, int S,
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
    // the partials of RSU slices in flight at once (a plain loop over s waited
    // for each slice's loads before issuing the next: S serial round trips)
    for (int s0 = 0; s0 < S; s0 += RSU) {
        float4 a[RSU][VPT], b[RSU][VPT];
#pragma unroll
        for (int j = 0; j < RSU; ++j) {
            const float4* pp = reinterpret_cast<const float4*>(part + ((size_t)min(s0 + j, S - 1) * M + m) * N);
#pragma unroll
            for (int i = 0; i < VPT; ++i) {
                const int idx = min(threadIdx.x + i * kBlock, nvec - 1);
                a[j][i] = pp[2 * idx];
                b[j][i] = pp[2 * idx + 1];
            }
        }
#pragma unroll
        for (int j = 0; j < RSU; ++j) {
            const float u = s0 + j < S ? 1.f : 0.f;  // branch-free: a branch let the loads sink to their uses
#pragma unroll
            for (int i = 0; i < VPT; ++i) {
                h[i][0] = fmaf(u, a[j][i].x, h[i][0]); h[i][1] = fmaf(u, a[j][i].y, h[i][1]);
                h[i][2] = fmaf(u, a[j][i].z, h[i][2]); h[i][3] = fmaf(u, a[j][i].w, h[i][3]);
                h[i][4] = fmaf(u, b[j][i].x, h[i][4]); h[i][5] = fmaf(u, b[j][i].y, h[i][5]);
                h[i][6] = fmaf(u, b[j][i].z, h[i][6]); h[i][7] = fmaf(u, b[j][i].w, h[i][7]);
            }
        }
    }
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            float yv[8], r[8];
            unpack8(pack8(h[i]), yv);
            unpack8(rv[i], r);
#pragma unroll
            for (int j = 0; j < 8; ++j) yv[j] += r[j];
            const uint4 packed = pack8(yv);
            rr[idx] = packed;
            unpack8(packed, h[i]);
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

// split-K reduction of the QKV projection + rotate-half RoPE on q and k, q
// written out, k / v appended to the KV cache (bf16, or KV8 fp8 e4m3) at
// (slot[t], :, pos[t], :) -- dmcp_kernels.hip::rope_kv_kernel over an LDS row
// of the bf16-rounded sum (what F.linear + rope_kv compute).
template <bool KV8>
__global__ __launch_bounds__(kBlock) void reduce_rope_kv_kernel(
    const float* __restrict__ part, int S, int M, const int32_t* __restrict__ pos, const int32_t* __restrict__ slot,
    const float2* __restrict__ cos_sin, uint16_t* __restrict__ q_out, void* __restrict__ k_cache,
    void* __restrict__ v_cache, int Hq, int Hkv, int D, int max_seq, int max_pos, int num_slots) {
    __shared__ uint4 rowbuf[8192 / 8];
    const int t = blockIdx.x;
    const int N = (Hq + 2 * Hkv) * D;
    const int nvec = N >> 3;
    for (int idx = threadIdx.x; idx < nvec; idx += kBlock) {
        float h[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        sum_slices8(part, S, M, t, N, idx, h);
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
    const int nunits = (Hq + Hkv) * quads;
    for (int uu = threadIdx.x; uu < nunits; uu += kBlock) {
        const int hh = uu / quads;
        const int d0 = (uu - hh * quads) * 4;
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
    const uint4* vsrc = rowbuf + (((Hq + Hkv) * D) >> 3);
    for (int uu = threadIdx.x; uu < vvec; uu += kBlock) {
        const int e = uu << 3;
        const int kh = e / D;
        const int d = e - kh * D;
        const size_t vofs = (((size_t)sl * Hkv + kh) * max_seq + p) * D + d;
        if constexpr (KV8)
            *reinterpret_cast<uint2*>(static_cast<uint8_t*>(v_cache) + vofs) = bf16x8_to_fp8x8(vsrc[uu]);
        else
            *reinterpret_cast<uint4*>(static_cast<uint16_t*>(v_cache) + vofs) = vsrc[uu];
    }
}

constexpr int kStages = 3;  // LDS ring stages (2 in flight while one is computed)
// dmcp_wgemm_set_aux: the weight stream's cache policy (0 default, 2 nt)
int g_wgemm_auxw = 0;

template <int NB, int MODE>
hipError_t launch_wgemm(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, int M, int N, int K, int S,
                        int mparts, int I, hipStream_t st, const uint32_t* masks = nullptr,
                        const int32_t* midx = nullptr, int n_masks = 0, int wwords = 0) {
    const int ntiles = (MODE == MODE_SWIGLU ? 2 * I : N) / NB;
    const int mrows = (((M + mparts - 1) / mparts) + 15) & ~15;
    const int mt = (mrows + 4 * 16 - 1) / (4 * 16);  // 16-row tiles per wave
    const bool full = ((mrows + 31) & ~31) > (mt - 1) * 64 + 32;  // staged rows: mt * 64, else mt * 64 - 32
    const dim3 grid((unsigned)(ntiles * S * mparts));
    const int ks = K / S;
#define DMCP_WG1(MT, MR)                                                                                        \
    do {                                                                                                        \
        if (g_wgemm_auxw == 2)                                                                                  \
            wgemm_kernel<NB, MT, MR, MODE, kStages, 2><<<grid, kBlock, 0, st>>>(                                \
                x, w, y, part, M, N, K, ks, S, ntiles, mparts, mrows, I, masks, midx, n_masks, wwords);         \
        else                                                                                                    \
            wgemm_kernel<NB, MT, MR, MODE, kStages><<<grid, kBlock, 0, st>>>(                                   \
                x, w, y, part, M, N, K, ks, S, ntiles, mparts, mrows, I, masks, midx, n_masks, wwords);         \
    } while (0)
#define DMCP_WG(MT)                  \
    do {                             \
        if (full)                    \
            DMCP_WG1(MT, MT * 64);   \
        else                         \
            DMCP_WG1(MT, MT * 64 - 32); \
    } while (0)
    switch (mt) {
        case 1: DMCP_WG(1); break;
        case 2: DMCP_WG(2); break;
        case 3: DMCP_WG(3); break;
        case 4: DMCP_WG(4); break;
        default: return hipErrorInvalidValue;
    }
#undef DMCP_WG
#undef DMCP_WG1
    return hipGetLastError();
}

}  // namespace

extern "C" {

// cache policy of the weight stream's LDS-DMA (0 or 2 = nt); returns the previous value
int dmcp_wgemm_set_aux(int aux) {
    const int old = g_wgemm_auxw;
    if (aux == 0 || aux == 2) g_wgemm_auxw = aux;
    return old;
}

// Plain / partial / SwiGLU weight-streaming GEMM.
//   mode 0: y[M, N] bf16 = x . w^T                        (S == 1)
//   mode 1: part[S, M, N] fp32 partials over K / S slices
//   mode 2: y[M, I] bf16 = silu(x . w[:I]^T) * (x . w[I:]^T)  (w = [gate; up] [2I, K], S == 1)
// Contract (checked by dmcp/ops/hip.py, guarded here): M in [1, 512],
// K % (64 S) == 0, N % 64 == 0 (mode 2: I % 64 == 0), rows / parts <= 256.
int dmcp_wgemm(const void* x, const void* w, void* y, void* part, int M, int N, int K, int S, int mparts, int mode,
               int I, void* stream) {
    if (M <= 0) return 0;
    if (!x || !w || M > 512 || S < 1 || mparts < 1 || K % (kKC * S) != 0 || (mode == 1 && !part) ||
        (mode != 1 && (!y || S != 1)) || (mode == 2 ? (I <= 0 || I % 64 != 0) : (N <= 0 || N % 64 != 0)) ||
        (((M + mparts - 1) / mparts + 15) & ~15) > 256)
        return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    auto xx = (const uint16_t*)x;
    auto ww = (const uint16_t*)w;
    auto yy = (uint16_t*)y;
    auto pp = (float*)part;
    // 64 weight rows per block (128 = 64 gate + 64 up for SwiGLU): 128-row
    // tiles for the plain / split-K forms measured slower at 78 and 320 rows
    // (4.80 vs 4.68 ms per fp8 step at 320, profiles/wgemm_r3.txt) -- the
    // halved X traffic does not pay for the doubled accumulators
    switch (mode) {
        case 0: return launch_wgemm<64, MODE_BF16>(xx, ww, yy, pp, M, N, K, S, mparts, 0, st);
        case 1: return launch_wgemm<64, MODE_PART>(xx, ww, yy, pp, M, N, K, S, mparts, 0, st);
        case 2: return launch_wgemm<128, MODE_SWIGLU>(xx, ww, yy, pp, M, 2 * I, K, S, mparts, I, st);
        default: return hipErrorInvalidValue;
    }
}

// LM head + grammar-masked greedy selection: ids[m] = argmax over the ids v
// allowed by mask row midx[m] (masks [n_masks, wwords] bitsets) of
// bf16(x[m] . w[v]); best: float2 workspace of (V / NB) * M pairs.  NB = 128
// vocabulary rows per block when V % 128 == 0 (fewer re-reads of x), else
// 64.  Contract: M in [1, 512], K % 64 == 0, V % 64 == 0, rows / part <= 256.
int dmcp_lm_head_argmax(const void* x, const void* w, const void* masks, const void* midx, int n_masks, int wwords,
                        void* best, void* ids, int M, int V, int K, int mparts, void* stream) {
    if (M <= 0) return 0;
    if (!x || !w || !masks || !best || !ids || M > 512 || n_masks < 1 || wwords < (V + 31) / 32 || mparts < 1 ||
        K % kKC != 0 || V <= 0 || V % 64 != 0 || (((M + mparts - 1) / mparts + 15) & ~15) > 256)
        return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    auto xx = (const uint16_t*)x;
    auto ww = (const uint16_t*)w;
    auto bb = (float*)best;
    auto mk = (const uint32_t*)masks;
    auto mi = (const int32_t*)midx;
    hipError_t e;
    int ntiles;
    if (V % 128 == 0) {
        ntiles = V / 128;
        e = launch_wgemm<128, MODE_ARGMAX>(xx, ww, nullptr, bb, M, V, K, 1, mparts, 0, st, mk, mi, n_masks, wwords);
    } else {
        ntiles = V / 64;
        e = launch_wgemm<64, MODE_ARGMAX>(xx, ww, nullptr, bb, M, V, K, 1, mparts, 0, st, mk, mi, n_masks, wwords);
    }
    if (e != hipSuccess) return e;
    argmax_pairs_kernel<<<(M + kBlock / kWave - 1) / (kBlock / kWave), kBlock, 0, st>>>(
        (const float2*)best, ntiles, M, (int32_t*)ids);
    return hipGetLastError();
}

// resid[M, N] += bf16(x . w^T); out = RMSNorm(resid) * g  (split-K GEMM +
// fused reduction; part: fp32 workspace of S * M * N).
int dmcp_wgemm_resid_norm(const void* x, const void* w, void* part, void* resid, const void* g, void* out, int M,
                          int K, int N, int S, int mparts, float eps, void* stream) {
    if (M <= 0) return 0;
    if (!resid || !g || !out || N % 8 != 0 || N > 8 * 4 * kBlock) return hipErrorInvalidValue;
    hipError_t e = (hipError_t)dmcp_wgemm(x, w, nullptr, part, M, N, K, S, mparts, 1, 0, stream);
    if (e != hipSuccess) return e;
    auto st = (hipStream_t)stream;
    const int vpt = (N / 8 + kBlock - 1) / kBlock;
    auto pp = (const float*)part;
    auto rr = (uint16_t*)resid;
    auto gg = (const uint16_t*)g;
    auto oo = (uint16_t*)out;
    if (vpt == 1) reduce_resid_norm_kernel<1><<<M, kBlock, 0, st>>>(pp, S, rr, gg, oo, M, N, eps);
    else if (vpt == 2) reduce_resid_norm_kernel<2><<<M, kBlock, 0, st>>>(pp, S, rr, gg, oo, M, N, eps);
    else reduce_resid_norm_kernel<4><<<M, kBlock, 0, st>>>(pp, S, rr, gg, oo, M, N, eps);
    return hipGetLastError();
}

// q_out[M, Hq, D] = RoPE(q); k / v appended to the caches; of qkv = x . w^T
// (w [(Hq + 2 Hkv) D, K]) -- F.linear + rope_kv in one GEMM + one reduction.
int dmcp_wgemm_rope_kv(const void* x, const void* w, void* part, const void* pos, const void* slot,
                       const void* cos_sin, void* q_out, void* k_cache, void* v_cache, int M, int K, int Hq, int Hkv,
                       int D, int max_seq, int max_pos, int num_slots, int kv8, int S, int mparts, void* stream) {
    if (M <= 0) return 0;
    const int N = (Hq + 2 * Hkv) * D;
    if (D % 16 != 0 || N > 8192 || !pos || !slot || !cos_sin || !q_out || !k_cache || !v_cache || max_pos <= 0)
        return hipErrorInvalidValue;
    hipError_t e = (hipError_t)dmcp_wgemm(x, w, nullptr, part, M, N, K, S, mparts, 1, 0, stream);
    if (e != hipSuccess) return e;
    auto st = (hipStream_t)stream;
    auto pp = (const float*)part;
    if (kv8)
        reduce_rope_kv_kernel<true><<<M, kBlock, 0, st>>>(pp, S, M, (const int32_t*)pos, (const int32_t*)slot,
                                                          (const float2*)cos_sin, (uint16_t*)q_out, k_cache, v_cache,
                                                          Hq, Hkv, D, max_seq, max_pos, num_slots);
    else
        reduce_rope_kv_kernel<false><<<M, kBlock, 0, st>>>(pp, S, M, (const int32_t*)pos, (const int32_t*)slot,
                                                           (const float2*)cos_sin, (uint16_t*)q_out, k_cache,
                                                           v_cache, Hq, Hkv, D, max_seq, max_pos, num_slots);
    return hipGetLastError();
}

// The split-K reductions alone, for partials written by another GEMM (the MX
// fp8 decode GEMM of pgemm.hip): resid += bf16(sum part); out = RMSNorm * g.
int dmcp_reduce_resid_norm(const void* part, int S, void* resid, const void* g, void* out, int M, int N, float eps,
                           void* stream) {
    if (M <= 0) return 0;
    if (!part || S < 1 || !resid || !g || !out || N % 8 != 0 || N > 8 * 4 * kBlock) return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    const int vpt = (N / 8 + kBlock - 1) / kBlock;
    auto pp = (const float*)part;
    auto rr = (uint16_t*)resid;
    auto gg = (const uint16_t*)g;
    auto oo = (uint16_t*)out;
    if (vpt == 1) reduce_resid_norm_kernel<1><<<M, kBlock, 0, st>>>(pp, S, rr, gg, oo, M, N, eps);
    else if (vpt == 2) reduce_resid_norm_kernel<2><<<M, kBlock, 0, st>>>(pp, S, rr, gg, oo, M, N, eps);
    else reduce_resid_norm_kernel<4><<<M, kBlock, 0, st>>>(pp, S, rr, gg, oo, M, N, eps);
    return hipGetLastError();
}

// ... and RoPE + q write + KV append of QKV partials [S, M, (Hq + 2 Hkv) D]
int dmcp_reduce_rope_kv(const void* part, int S, const void* pos, const void* slot, const void* cos_sin, void* q_out,
                        void* k_cache, void* v_cache, int M, int Hq, int Hkv, int D, int max_seq, int max_pos,
                        int num_slots, int kv8, void* stream) {
    if (M <= 0) return 0;
    if (!part || S < 1 || D % 16 != 0 || (Hq + 2 * Hkv) * D > 8192 || !pos || !slot || !cos_sin || !q_out ||
        !k_cache || !v_cache || max_pos <= 0)
        return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    auto pp = (const float*)part;
    if (kv8)
        reduce_rope_kv_kernel<true><<<M, kBlock, 0, st>>>(pp, S, M, (const int32_t*)pos, (const int32_t*)slot,
                                                          (const float2*)cos_sin, (uint16_t*)q_out, k_cache, v_cache,
                                                          Hq, Hkv, D, max_seq, max_pos, num_slots);
    else
        reduce_rope_kv_kernel<false><<<M, kBlock, 0, st>>>(pp, S, M, (const int32_t*)pos, (const int32_t*)slot,
                                                           (const float2*)cos_sin, (uint16_t*)q_out, k_cache,
                                                           v_cache, Hq, Hkv, D, max_seq, max_pos, num_slots);
    return hipGetLastError();
}

}  // extern "C"
