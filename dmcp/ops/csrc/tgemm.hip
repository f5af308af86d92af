// Large-tile decode GEMM for steps of 257-1024 rows (gfx950 / MI355X, CDNA4):
//
//   Y[M, N] = X[M, K] . W[N, K]^T      bf16 in, fp32 accumulate
//
// The decode step's row count passes 512 whenever the engine's jump-forward
// rows fill its spare capacity (max_rows = 768 at 512 KV slots).  There the
// projections are compute-bound (a 640-row step is ~1.2 TFLOP over ~2 GB of
// weights) and wgemm.hip's 64-128-row weight tiles re-stage the activation
// rows once per tile: its staged bytes grow with M x N / NB.  This kernel
// keeps wgemm's building blocks (LDS-DMA ring with a counted vmcnt + raw
// barrier per stage, C^T = W . X^T tiles on v_mfma_f32_16x16x32_bf16, the M
// parts of one weight tile on one XCD, fused epilogues) with a 4x larger
// weight tile:
//
//   * a block owns 256 weight rows (SwiGLU: 128 gate + the 128 up rows of the
//     same intermediate columns) x 32 XT activation rows (XT = 2..8), i.e. up
//     to 256 x 256 outputs, over 8 waves (two per SIMD): 4 weight quarters x
//     2 M halves, each 64 weight rows x 16 XT rows (4 A x XT B fragments,
//     16 XT accumulators) -- near-square wave tiles keep the LDS fragment
//     reads (the CU's LDS array served ~90 % of its bandwidth to 128 x 32
//     wave tiles' redundant reads) at (64 + 16 XT) rows per wave and k step.
//     The X rows go in 32-row steps (round 6; 64 before): a 153-row M part
//     stages 160 rows, and (256 + 160) x 128 B stages fit THREE in the LDS
//     where 192 rows fit two -- one stage more in flight;
//   * waves 4-7 (one per SIMD) also issue the block's LDS-DMA: an LDS-DMA
//     instruction holds its wave's issue for ~60-185 cycles
//     (MI355X_MICROARCH.md, cycle constants), and with one wave per SIMD doing
//     both, the 8 pieces per stage ran in series with its MFMAs (v1 of this
//     kernel: 45 % of MFMA time at 1,024 rows); now the SIMD partner keeps
//     issuing MFMAs meanwhile;
//   * 32-deep K stages ([rows][4 x 16 B] images, 16-row 1-KiB LDS-DMA
//     pieces) in a 5-6-stage ring filling the CU's LDS (tstages);
//   * chunk j of row r sits in slot j ^ ((4 - (r >> 2)) & 3): the 16 lanes of
//     each ds_read_b128 group of the 16x16x32 operand layout (lane (l16, g):
//     row l16, chunk g) cover all 64 banks;
//   * split-K slices of whole stages (any count: the last slice may be
//     shorter) for the narrow projections; the fp32 partials are reduced by
//     wgemm.hip's fused consumers (RoPE + KV append, residual + RMSNorm);
//   * MODE_ARGMAX: the LM head + grammar-masked greedy selection (per block
//     and row one (max, id) pair per 64 vocabulary ids, a per-row
//     reduction kernel selects), no [M, V] logits.
#include "dmcp_common.hpp"

namespace {

// K per LDS stage: 64 (128-B image rows, full cache lines per DMA lane
// group) or 32 (64-B rows: each 128-B line is fetched twice, in two stages)
constexpr int TKC_DEFAULT = 64;
// ring stages: as many stages as fit the CU's 160 KiB of LDS (capped at 6;
// RES bytes reserved)
template <int XT, int KC, int CAP = 6, int RES = 0>
constexpr int tstages() {
    return (160 * 1024 - RES) / ((256 + 32 * XT) * KC * 2) < CAP ? (160 * 1024 - RES) / ((256 + 32 * XT) * KC * 2)
                                                                 : CAP;
}

// s_waitcnt vmcnt(n * GL) for a runtime n in [0, 5] (the count is an immediate)
// (counts past the 6-bit field are never reached: n <= stages - 2, and a
// ring of that many stages of GL pieces fits the counter; they compile to
// the full wait)
template <int K>
__device__ __forceinline__ void wait_vm_k() {
    if constexpr (K <= 63) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(K) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
template <int GL>
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: wait_vm_k<GL>(); break;
        case 2: wait_vm_k<2 * GL>(); break;
        case 3: wait_vm_k<3 * GL>(); break;
        case 4: wait_vm_k<4 * GL>(); break;
        default: wait_vm_k<5 * GL>(); break;
    }
}
constexpr int TNB = 256;  // weight rows per block
constexpr int TTH = 512;  // threads per block: 8 waves, two per SIMD
constexpr int TM_BF16 = 0, TM_PART = 1, TM_SWIGLU = 2, TM_ARGMAX = 3;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float tsilu(float g) { return g / (1.f + __expf(-g)); }

__device__ __forceinline__ void tglds16(const void* src, uint4* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// slot of logical 16-B chunk j of image row r: 64-B rows (4 chunks): j ^
// ((4 - (r >> 2)) & 3); 128-B rows (8 chunks): j ^ (r & 7) -- either way the
// 16 lanes of each ds_read_b128 group of the 16x16x32 operand layout (lane
// (l16, g): row l16, chunk g of the k step) cover all 64 banks
template <int KC>
__device__ __forceinline__ int tslot(int j, int r) {
    if constexpr (KC == 32) return j ^ ((4 - (r >> 2)) & 3);
    else return j ^ (r & 7);
}

// s_waitcnt vmcnt(n) for a runtime n in [0, 63] (the count is an immediate)
constexpr int kVmMax = 63;
__device__ __forceinline__ void wait_vm_rt(int n) {
    switch (n) {
#define DMCP_VMC(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
        DMCP_VMC(0) DMCP_VMC(1) DMCP_VMC(2) DMCP_VMC(3) DMCP_VMC(4) DMCP_VMC(5) DMCP_VMC(6) DMCP_VMC(7) DMCP_VMC(8) DMCP_VMC(9) DMCP_VMC(10) DMCP_VMC(11) DMCP_VMC(12) DMCP_VMC(13) DMCP_VMC(14) DMCP_VMC(15) DMCP_VMC(16) DMCP_VMC(17) DMCP_VMC(18) DMCP_VMC(19) DMCP_VMC(20) DMCP_VMC(21) DMCP_VMC(22) DMCP_VMC(23) DMCP_VMC(24) DMCP_VMC(25) DMCP_VMC(26) DMCP_VMC(27) DMCP_VMC(28) DMCP_VMC(29) DMCP_VMC(30) DMCP_VMC(31) DMCP_VMC(32) DMCP_VMC(33) DMCP_VMC(34) DMCP_VMC(35) DMCP_VMC(36) DMCP_VMC(37) DMCP_VMC(38) DMCP_VMC(39) DMCP_VMC(40) DMCP_VMC(41) DMCP_VMC(42) DMCP_VMC(43) DMCP_VMC(44) DMCP_VMC(45) DMCP_VMC(46) DMCP_VMC(47) DMCP_VMC(48) DMCP_VMC(49) DMCP_VMC(50) DMCP_VMC(51) DMCP_VMC(52) DMCP_VMC(53) DMCP_VMC(54) DMCP_VMC(55) DMCP_VMC(56) DMCP_VMC(57) DMCP_VMC(58) DMCP_VMC(59) DMCP_VMC(60) DMCP_VMC(61) DMCP_VMC(62)
#undef DMCP_VMC
        default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
    }
}

// PROBE (dmcp_tgemm_probe only; diagnostics of scripts/bench_tgemm.py --probe):
// 1 = the K loop issues no refill DMAs (MFMA + LDS reads + barriers on stale
// stages), 2 = no fragment reads / MFMAs (the DMA ring alone)
//
// PF > 0: L2 prefetch of the weight stream PF stages ahead of the ring.  At
// XT = 6-8 only two stages fit the LDS, so one 56-64 KB stage is in flight
// per CU and the ring runs at that stage's HBM latency (~31 KB/us per CU
// measured on the LM head, half the L2-fed rate); a 4-byte LDS-DMA
// (global_load_lds_dword: no register, a 256-B scratch slot of LDS) per
// 128-B weight line, issued PF stages before its refill, turns the refill
// into an L2 hit.  Waves 0-3 (not the loaders) issue them: vector memory
// loads complete in order, so a prefetch in a loader's queue would hold
// back that loader's counted wait for the next stage by a full HBM latency.
// MEASURED SLOWER at every distance (probes 257-262: +5-20 % on the
// projections, +9-35 % on the LM head, worse with depth;
// profiles/tgemm_l2_prefetch_ab_r5.jsonl): the refills are not waiting on
// HBM latency.  Diagnostic only; production launches use PF = 0.
template <int XT, int MODE, int PROBE = 0, int KC = TKC_DEFAULT, int CAP = 6, int PF = 0>
__global__ __launch_bounds__(TTH) __attribute__((amdgpu_waves_per_eu(2, 2))) void tgemm_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y, float* __restrict__ part,
    int M, int N, int K, int cps, int S, int ntiles, int mparts, int mrows, int I, const uint32_t* __restrict__ masks,
    const int32_t* __restrict__ midx, int n_masks, int wwords) {
    constexpr int NF = TNB / 64;       // A fragments per wave (16 weight rows each): a quarter of the tile's rows
    constexpr int RCH = KC / 8;        // 16-B chunks per image row
    constexpr int PR = 64 / RCH;       // image rows per 1-KiB LDS-DMA piece
    constexpr int MR = 32 * XT;        // staged X rows (XT B fragments of 16 rows per wave, 2 M halves)
    constexpr int WI = TNB / PR / 4;   // pieces per loader wave per stage: weights
    constexpr int XI = MR / PR / 4;    //                                   X rows
    constexpr int GL = WI + XI;        // LDS-DMA instructions per loader wave per stage
    constexpr int WCH = TNB * RCH;     // 16-B chunks of a stage's weight image
    constexpr int SCH = WCH + MR * RCH;  // ... plus the X image
    constexpr int PFB = PF > 0 ? 1024 : 0;  // prefetch scratch: 256 B per loader wave
    constexpr int TST = tstages<XT, KC, CAP, PFB>();
    static_assert(MR % (PR * 4) == 0, "X pieces per loader wave");
    static_assert(TST >= 2 && TST * SCH * 16 + PFB <= 160 * 1024, "LDS ring");
    __shared__ uint4 lds[TST * SCH + PFB / 16];   // ONE shared array (cdna_hip_programming.md §5 item 4a)

    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    // waves 0-3 and 4-7 each cover the 4 SIMDs once: waves 4-7 also issue the
    // block's LDS-DMA (one loader per SIMD), so while a loader waits on its
    // DMA issue its SIMD partner keeps the matrix core busy
    const bool loader = wv >= 4;
    const int lw = wv & 3;                 // loader index
    const int wn = wv & 3, wm = wv >> 2;   // weight quarter (64 rows) x M half (16 XT rows)
    const int l16 = lane & 15, g = lane >> 4;
    // block -> (weight tile nt, K slice s, M part mp): the M parts of one
    // (nt, s) unit share blockIdx % 8 (one XCD) and consecutive dispatch slots
    const int units = ntiles * S;
    int u, mp;
    if ((units & 7) == 0) {
        const int j = blockIdx.x >> 3;
        u = (j / mparts) * 8 + (blockIdx.x & 7);
        mp = j % mparts;
    } else {
        // XCD-contiguous ranges (bijective for any grid; blocks are dealt
        // round-robin over the 8 XCDs): a unit's M parts are consecutive in
        // one XCD's range, so its weight tile is read once from HBM / MALL
        // and hit in that XCD's L2 by the other parts (the LM head: 501
        // units, whose parts had landed on three different XCDs)
        const int nblk = units * mparts, b = blockIdx.x;
        const int xcd = b & 7, q8 = nblk >> 3, r8 = nblk & 7;
        const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
        u = L / mparts;
        mp = L % mparts;
    }
    const int nt = u % ntiles, s = u / ntiles;
    const int chunks_all = K / KC;
    const int cbeg = s * cps;
    const int chunks = min(chunks_all, cbeg + cps) - cbeg;  // > 0 (host contract)
    const int m_lo = mp * mrows;
    const int m_hi = min(M, m_lo + mrows);
    const int mw = wm * (XT * 16);
    int mtv = (m_hi - m_lo - mw + 15) / 16;  // valid 16-row tiles of this wave (wave-uniform)
    mtv = max(0, min(XT, mtv));

    const int n0 = nt * TNB;
    const int n0h = nt * (TNB / 2);
    // weight row of image row r.  SwiGLU: each 64-row quarter holds 32 gate
    // rows then the 32 up rows of the same intermediate columns, so a wave's
    // gate fragment f and up fragment f + NF / 2 meet in one lane
    auto wrow = [&](int r) -> int {
        if constexpr (MODE == TM_SWIGLU) {
            const int h = r >> 6, i = r & 63;
            return (i < 32 ? 0 : I) + n0h + 32 * h + (i & 31);
        } else {
            return n0 + r;
        }
    };
    // LDS-DMA sources: lane L of a piece fills image row base + L / RCH, slot
    // L % RCH with logical chunk tslot(L % RCH, row) (an involution)
    const uint16_t* wsrc[WI];
    const uint16_t* xsrc[XI];
#pragma unroll
    for (int i = 0; i < WI; ++i) {
        const int r = (lw * WI + i) * PR + lane / RCH;
        wsrc[i] = w + (size_t)wrow(r) * K + (size_t)cbeg * KC + tslot<KC>(lane % RCH, r) * 8;
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {
        const int r = (lw * XI + i) * PR + lane / RCH;
        xsrc[i] = x + (size_t)min(m_lo + r, M - 1) * K + (size_t)cbeg * KC + tslot<KC>(lane % RCH, r) * 8;
    }
    // prefetch: lane of wave lw (< 4) -> weight row 64 lw + lane, one 4-B
    // read of its 128-B line of the stage
    const uint16_t* pfsrc = w + (size_t)wrow(64 * lw + lane) * K + (size_t)cbeg * KC;
    auto prefetch = [&](int c) {
        if constexpr (PF > 0)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(pfsrc + c * KC),
                                             (__attribute__((address_space(3))) void*)(lds + TST * SCH + 16 * lw), 4,
                                             0, 0);
    };
    auto issue = [&](int c, int slot) {
        uint4* base = lds + slot * SCH;
#pragma unroll
        for (int i = 0; i < WI; ++i) tglds16(wsrc[i] + c * KC, base + (lw * WI + i) * 64);
#pragma unroll
        for (int i = 0; i < XI; ++i) tglds16(xsrc[i] + c * KC, base + WCH + (lw * XI + i) * 64);
    };

    f32x4_t acc[NF][XT];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int t = 0; t < XT; ++t) acc[f][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // Per stage KC / 32 k steps of XT X fragments and NF weight fragments
    // (this wave's 64 weight rows) and NF x XT MFMAs; the next k step's
    // reads are threaded between the current one's MFMAs (pinned: the
    // scheduler would sink each read to its use).
    constexpr int KS = KC / 32;
    auto compute = [&](const uint4* st) {
        const uint4* wl = st;
        const uint4* xl = st + WCH;
        bf16x8_t a[KS][NF], b[KS][XT];
        auto load = [&](int kk) {
#pragma unroll
            for (int t = 0; t < XT; ++t) {
                const int r = mw + 16 * t + l16;
                b[kk][t] = as_bf16x8(xl[r * RCH + tslot<KC>(4 * kk + g, r)]);
            }
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int r = 64 * wn + 16 * f + l16;
                a[kk][f] = as_bf16x8(wl[r * RCH + tslot<KC>(4 * kk + g, r)]);
            }
        };
        auto mma = [&](int kk) {
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int t = 0; t < XT; ++t)
                    acc[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][f], b[kk][t], acc[f][t], 0, 0, 0);
        };
        load(0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            if (kk + 1 < KS) load(kk + 1);
            mma(kk);
            if (kk + 1 < KS) {
                constexpr int NR = NF + XT, NM = NF * XT, RM = NM / NR > 0 ? NM / NR : 1;
#pragma unroll
                for (int i = 0; i < NR; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one DS read
                    __builtin_amdgcn_sched_group_barrier(0x008, RM, 0);  // RM MFMAs
                }
                __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);      // the rest
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    };

    // TST-stage ring, TST - 1 stages in flight: a loader waits for its pieces
    // of stage c (counted vmcnt: the newer stages stay in flight), one raw
    // barrier (stage c landed for every wave; every wave done with stage
    // c - 1, the slot about to be refilled), the loaders refill it with stage
    // c + TST - 1, everyone computes stage c.  No __syncthreads() in the loop.
    // With PF, waves 0-3 prefetch stages TST - 1 .. TST - 2 + PF up front and
    // stage c + TST - 1 + PF in iteration c (they never wait in the loop).
    if (loader) {
#pragma unroll
        for (int j = 0; j < TST - 1; ++j)
            if (j < chunks) issue(j, j);
    } else if constexpr (PF > 0) {
#pragma unroll
        for (int q = TST - 1; q < TST - 1 + PF; ++q)
            if (q < chunks) prefetch(q);
    }
    for (int c = 0; c < chunks; ++c) {
        if (loader) {
            if constexpr ((PROBE & 1) != 0) wait_vm<GL>(0);
            else wait_vm<GL>(min(TST - 2, chunks - 1 - c));
        }
        asm volatile("s_barrier" ::: "memory");
        if ((PROBE & 1) == 0) {
            if (loader) {
                if (c + TST - 1 < chunks) issue(c + TST - 1, (c + TST - 1) % TST);
            } else if (PF > 0 && c + TST - 1 + PF < chunks) {
                prefetch(c + TST - 1 + PF);
            }
        }
        if constexpr ((PROBE & 2) == 0) compute(lds + (c % TST) * SCH);
    }
    if constexpr (PF > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the prefetches landed

    // epilogue: lane (l16, g) holds Y[row m_lo + mw + 16t + l16][col c0 + 16f + 4g + i]
    // with c0 = n0 + 64 wn (SwiGLU: intermediate column n0h + 32 wn + 16f + 4g + i of f < NF / 2)
    const int c0 = n0 + 64 * wn;
#pragma unroll
    for (int t = 0; t < XT; ++t) {
        if (t >= mtv) continue;
        const int m = m_lo + mw + 16 * t + l16;
        if constexpr (MODE == TM_ARGMAX) {
            float bv = -INFINITY;
            int bi = 0x7fffffff;
            if (m < m_hi) {
                int mr = midx ? midx[m] : 0;
                mr = mr < 0 ? 0 : (mr >= n_masks ? n_masks - 1 : mr);
                const uint32_t* mrow = masks + (size_t)mr * wwords + (c0 >> 5);
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const uint32_t word = mrow[(16 * f + 4 * g) >> 5];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int c = 16 * f + 4 * g + i;
                        if ((word >> (c & 31)) & 1u) {
                            const float v = bf2f(f2bf(acc[f][t][i]));
                            if (v > bv) { bv = v; bi = c0 + c; }  // columns ascend: strict > keeps the lowest
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
            // one (max, id) pair per 64-id quarter tile and row
            if (m < m_hi && g == 0)
                reinterpret_cast<float2*>(part)[(size_t)(4 * nt + wn) * M + m] = make_float2(bv, __int_as_float(bi));
            continue;
        }
        if (m >= m_hi) continue;
        if constexpr (MODE == TM_SWIGLU) {
#pragma unroll
            for (int f = 0; f < NF / 2; ++f) {
                float o[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {  // gate / up rounded to bf16 as the unfused GEMM output is
                    const float gg = bf2f(f2bf(acc[f][t][i])), uu = bf2f(f2bf(acc[f + NF / 2][t][i]));
                    o[i] = tsilu(gg) * uu;
                }
                *reinterpret_cast<uint2*>(y + (size_t)m * I + n0h + 32 * wn + 16 * f + 4 * g) = pack4(o);
            }
        } else if constexpr (MODE == TM_PART) {
            float* dst = part + ((size_t)s * M + m) * N + c0 + 4 * g;
#pragma unroll
            for (int f = 0; f < NF; ++f)
                *reinterpret_cast<float4*>(dst + 16 * f) =
                    make_float4(acc[f][t][0], acc[f][t][1], acc[f][t][2], acc[f][t][3]);
        } else {
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const float o[4] = {acc[f][t][0], acc[f][t][1], acc[f][t][2], acc[f][t][3]};
                *reinterpret_cast<uint2*>(y + (size_t)m * N + c0 + 16 * f + 4 * g) = pack4(o);
            }
        }
    }
}


// Register-weight variant (diagnostic: dmcp_tgemm_probe 64-66 / 129-130
// only).  MEASURED SLOWER and not used: 1.2-1.4x tgemm_kernel's time at
// 610-1,024 rows on every projection; its weight loads alone (probe 66)
// take 1.6-1.75x the LDS-DMA ring alone (probe 2) for the same bytes
// (profiles/tgemm_regweights_ab_r5.jsonl) -- consistent with
// MI355X_MICROARCH.md's gather table (register staging and LDS-DMA read
// at the same per-CU rate): the two paths share one per-CU ingest, and
// the MFMA operand layout's 16 rows x 64 B per load instruction costs
// more than the DMA's 8 rows x 128 B pieces.  The design, for the record:
//
// tgemm_kernel's probes put it at the CU's LDS-DMA ingest (~60 KB/us per CU:
// DMA alone ~ the whole kernel; MI355X_MICROARCH.md's ring-gemm measured 68
// GB/s per CU for the same path), with half of the staged bytes weights that
// one wave per M half reads back.  Here each of the 8 waves owns 32 weight
// rows (2 A fragments) x every staged X row (4 MT B fragments) and loads its
// weight fragments straight into VGPRs with plain 16-B global loads in the
// MFMA operand layout (lane (l16, g): row l16, k chunk g of the k step; 16
// rows x 64 contiguous bytes per instruction), D stages ahead in a rotating
// register ring; only the X rows go through the LDS-DMA ring, issued by all
// 8 waves.  Two memory paths per CU instead of one, and half the LDS-DMA.
// The K loop is branch-free (a guarded MFMA or DMA would leave the
// compiler's wait insertion a join where it falls back to vmcnt(0), which
// drains the register ring).
//
// Per stage c every wave: counted vmcnt (its X pieces and weight loads of
// stage c landed; everything newer stays in flight), raw barrier (every
// wave's pieces of stage c landed, every wave done with stage c - 1), X
// pieces of stage c + TST - 1 into the freed slot, weights of stage c + D
// into register buffer (c + D) % (D + 1), then compute stage c.
template <int MT, int MODE, int PROBE = 0, int D = 3, int KC = TKC_DEFAULT, int CAP = 6>
__global__ __launch_bounds__(TTH) __attribute__((amdgpu_waves_per_eu(2, 2))) void tgemm_r_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y, float* __restrict__ part,
    int M, int N, int K, int cps, int S, int ntiles, int mparts, int mrows, int I, const uint32_t* __restrict__ masks,
    const int32_t* __restrict__ midx, int n_masks, int wwords) {
    constexpr int NF = 2;               // A fragments per wave: 32 weight rows
    constexpr int XT = 4 * MT;          // B fragments per wave: every staged X row
    constexpr int RCH = KC / 8;         // 16-B chunks per image row
    constexpr int PR = 64 / RCH;        // image rows per 1-KiB LDS-DMA piece
    constexpr int MR = 64 * MT;         // staged X rows
    constexpr int XI = MR / PR / 8;     // X pieces per wave per stage
    constexpr int KS = KC / 32;         // k steps per stage
    constexpr int WL = NF * KS;         // weight loads per wave per stage
    constexpr int SCH = MR * RCH;       // 16-B chunks of a stage's X image
    constexpr int TST = (160 * 1024) / (SCH * 16) < CAP ? (160 * 1024) / (SCH * 16) : CAP;
    static_assert(TST >= 2 && TST - 1 >= D && XI >= 1, "ring");
    static_assert((D - 1) * (XI + WL) <= kVmMax, "counted vmcnt");
    static_assert(MODE == TM_PART, "diagnostic kernel: fp32 partials only");
    __shared__ uint4 lds[TST * SCH];

    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    const int l16 = lane & 15, g = lane >> 4;
    const int units = ntiles * S;
    int u, mp;
    if ((units & 7) == 0) {
        const int j = blockIdx.x >> 3;
        u = (j / mparts) * 8 + (blockIdx.x & 7);
        mp = j % mparts;
    } else {
        // XCD-contiguous ranges (bijective for any grid; blocks are dealt
        // round-robin over the 8 XCDs): a unit's M parts are consecutive in
        // one XCD's range, so its weight tile is read once from HBM / MALL
        // and hit in that XCD's L2 by the other parts (the LM head: 501
        // units, whose parts had landed on three different XCDs)
        const int nblk = units * mparts, b = blockIdx.x;
        const int xcd = b & 7, q8 = nblk >> 3, r8 = nblk & 7;
        const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
        u = L / mparts;
        mp = L % mparts;
    }
    const int nt = u % ntiles, s = u / ntiles;
    const int chunks_all = K / KC;
    const int cbeg = s * cps;
    const int chunks = min(chunks_all, cbeg + cps) - cbeg;  // > 0 (host contract)
    const int m_lo = mp * mrows;
    const int m_hi = min(M, m_lo + mrows);
    const int rows = m_hi - m_lo;
    const int mtv = __builtin_amdgcn_readfirstlane(min(XT, (rows + 15) / 16));  // 16-row tiles computed

    const int n0 = nt * TNB;
    auto wrow = [&](int r) -> int { return n0 + r; };
    const uint4* wp[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f)
        wp[f] = reinterpret_cast<const uint4*>(w + (size_t)wrow(32 * wv + 16 * f + l16) * K + (size_t)cbeg * KC) + g;
    const uint16_t* xsrc[XI];
#pragma unroll
    for (int i = 0; i < XI; ++i) {
        const int r = (wv * XI + i) * PR + lane / RCH;
        xsrc[i] = x + (size_t)min(m_lo + r, M - 1) * K + (size_t)cbeg * KC + tslot<KC>(lane % RCH, r) * 8;
    }
    auto issue_x = [&](int c, int slot) {
        uint4* base = lds + slot * SCH;
#pragma unroll
        for (int i = 0; i < XI; ++i)
            tglds16(xsrc[i] + c * KC, base + (wv * XI + i) * 64);
    };
    // the weight loads are inline asm: the compiler's wait insertion loses
    // count of builtin loads at the unrolled loop's back edge and drains the
    // whole ring (vmcnt(0)) there; their completion is the counted wait at
    // the top of each stage, after which `pin` hands the registers to the
    // compiler as defined
    u32x4_t wb[D + 1][WL];
    auto load_w = [&](u32x4_t (&dst)[WL], int c) {
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst[f * KS + kk]) : "v"(wp[f] + c * RCH + 4 * kk)
                             : "memory");
    };
    auto pin = [&](u32x4_t (&r)[WL]) {
#pragma unroll
        for (int i = 0; i < WL; ++i) asm volatile("" : "+v"(r[i]));
    };

    f32x4_t acc[NF][XT];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int t = 0; t < XT; ++t) acc[f][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // per k step: the B fragments of the computed tiles from LDS in groups of
    // GB, group q + 1's reads issued before group q's MFMAs (A from the
    // register ring); 2 GB fragments live, not XT
    constexpr int GB = XT < 4 ? XT : 4;
    constexpr int NQ = XT / GB;
    auto compute = [&](const uint4* xl, const u32x4_t (&a)[WL]) {
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            bf16x8_t b[2][GB];
            auto rd = [&](int q) {
#pragma unroll
                for (int e = 0; e < GB; ++e) {
                    const int r = 16 * (q * GB + e) + l16;
                    b[q & 1][e] = as_bf16x8(xl[r * RCH + tslot<KC>(4 * kk + g, r)]);
                }
            };
            rd(0);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                if (q + 1 < NQ) rd(q + 1);
#pragma unroll
                for (int e = 0; e < GB; ++e)
#pragma unroll
                    for (int f = 0; f < NF; ++f)
                        acc[f][q * GB + e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8_t, a[f * KS + kk]), b[q & 1][e], acc[f][q * GB + e], 0, 0, 0);
            }
        }
    };

    // vm operations this wave issued after its weight loads of stage c (they
    // and everything older, incl. the X pieces of stage c, must have landed)
    auto pending_after = [&](int c) -> int {
        int n = 0;
        if (c < D) n += WL * (min(D, chunks) - 1 - c);  // the prologue's later weight stages
        for (int i = max(0, c - D + 1); i < c; ++i)     // the loop iterations since
            n += (i + TST - 1 < chunks ? XI : 0) + (i + D < chunks ? WL : 0);
        return n;
    };

#pragma unroll
    for (int j = 0; j < TST - 1; ++j)
        if (j < chunks) issue_x(j, j);
#pragma unroll
    for (int j = 0; j < D; ++j)
        if (j < chunks) load_w(wb[j], j);
    for (int c0 = 0; c0 < chunks; c0 += D + 1) {
#pragma unroll
        for (int jj = 0; jj <= D; ++jj) {
            const int c = c0 + jj;
            if (c < chunks) {
                if constexpr ((PROBE & 1) != 0) wait_vm_rt(0);
                else wait_vm_rt(pending_after(c));
                pin(wb[jj]);
                asm volatile("s_barrier" ::: "memory");
                if constexpr ((PROBE & 1) == 0) {
                    if (c + TST - 1 < chunks) issue_x(c + TST - 1, (c + TST - 1) % TST);
                    if (c + D < chunks) load_w(wb[(jj + D) % (D + 1)], c + D);
                }
                if constexpr ((PROBE & 2) == 0) compute(lds + (c % TST) * SCH, wb[jj]);
            }
        }
    }
    // every weight load landed (the last stage waited for all of them): no
    // asm load may still write a register the epilogue reuses
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // epilogue: lane (l16, g) holds Y[row m_lo + 16t + l16][col n0 + 32 wv + 16f + 4g + i]
    const int c0 = n0 + 32 * wv;
#pragma unroll
    for (int t = 0; t < XT; ++t) {
        const int m = m_lo + 16 * t + l16;
        if (t >= mtv || m >= m_hi) continue;
        float* dst = part + ((size_t)s * M + m) * N + c0 + 4 * g;
#pragma unroll
        for (int f = 0; f < NF; ++f)
            *reinterpret_cast<float4*>(dst + 16 * f) = make_float4(acc[f][t][0], acc[f][t][1], acc[f][t][2], acc[f][t][3]);
    }
}

template <int MODE, int PROBE = 0, int KC = TKC_DEFAULT, int CAP = 6, int PF = 0>
hipError_t launch_tgemm(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, int M, int N, int K, int S,
                        int mparts, int I, hipStream_t st, const uint32_t* masks, const int32_t* midx, int n_masks,
                        int wwords) {
    const int ntiles = (MODE == TM_SWIGLU ? 2 * I : N) / TNB;
    const int mrows = (((M + mparts - 1) / mparts) + 15) & ~15;
    // staged X rows in 32-row steps (>= 64); 32-deep stages (probes) in 64-row steps
    int xt = (mrows + 31) / 32;
    xt = xt < 2 ? 2 : xt;
    if (KC == 32) xt = (xt + 1) & ~1;
    const int chunks = K / KC;
    const int cps = (chunks + S - 1) / S;
    const dim3 grid((unsigned)(ntiles * S * mparts));
#define DMCP_TG(XT)                                                                                                 \
    tgemm_kernel<XT, MODE, PROBE, KC, CAP, PF><<<grid, TTH, 0, st>>>(x, w, y, part, M, N, K, cps, S, ntiles, mparts, mrows, I, masks, \
                                                    midx, n_masks, wwords)
    if constexpr (KC == 32) {
        switch (xt) {
            case 2: DMCP_TG(2); break;
            case 4: DMCP_TG(4); break;
            case 6: DMCP_TG(6); break;
            case 8: DMCP_TG(8); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (xt) {
            case 2: DMCP_TG(2); break;
            case 3: DMCP_TG(3); break;
            case 4: DMCP_TG(4); break;
            case 5: DMCP_TG(5); break;
            case 6: DMCP_TG(6); break;
            case 7: DMCP_TG(7); break;
            case 8: DMCP_TG(8); break;
            default: return hipErrorInvalidValue;
        }
    }
#undef DMCP_TG
    return hipGetLastError();
}

template <int MODE, int PROBE = 0, int D = 3>
hipError_t launch_tgemm_r(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, int M, int N, int K, int S,
                          int mparts, int I, hipStream_t st, const uint32_t* masks, const int32_t* midx, int n_masks,
                          int wwords) {
    const int ntiles = (MODE == TM_SWIGLU ? 2 * I : N) / TNB;
    const int mrows = (((M + mparts - 1) / mparts) + 15) & ~15;
    const int mt = (mrows + 63) / 64;
    const int chunks = K / TKC_DEFAULT;
    const int cps = (chunks + S - 1) / S;
    const dim3 grid((unsigned)(ntiles * S * mparts));
#define DMCP_TG(MT)                                                                                          \
    tgemm_r_kernel<MT, MODE, PROBE, D><<<grid, TTH, 0, st>>>(x, w, y, part, M, N, K, cps, S, ntiles, mparts, \
                                                             mrows, I, masks, midx, n_masks, wwords)
    switch (mt) {
        case 1: DMCP_TG(1); break;
        case 2: DMCP_TG(2); break;
        case 3: DMCP_TG(3); break;
        case 4: DMCP_TG(4); break;
        default: return hipErrorInvalidValue;
    }
#undef DMCP_TG
    return hipGetLastError();
}

}  // namespace

extern "C" {

// Large-tile GEMM.
//   mode 0: y[M, N] bf16 = x . w^T                              (S == 1)
//   mode 1: part[S, M, N] fp32 partials over S K slices of ceil(K / 64 / S) stages
//   mode 2: y[M, I] bf16 = silu(x . w[:I]^T) * (x . w[I:]^T)     (w = [gate; up] [2I, K], S == 1)
//   mode 3: ids[M] = masked argmax of bf16(x . w^T) (w [V = N, K]; part: float2 workspace of N / 64 * M pairs;
//           masks [n_masks, wwords], midx [M]; S == 1)
// Contract (checked by dmcp/ops/hip.py, guarded here): K % 64 == 0, N % 256 == 0 (mode 2: I % 128 == 0),
// rows per M part <= 256, every K slice non-empty.
int dmcp_tgemm(const void* x, const void* w, void* y, void* part, int M, int N, int K, int S, int mparts, int mode,
               int I, const void* masks, const void* midx, int n_masks, int wwords, void* ids, void* stream) {
    if (M <= 0) return 0;
    const int chunks = K / TKC_DEFAULT;
    if (!x || !w || S < 1 || mparts < 1 || K <= 0 || K % TKC_DEFAULT != 0 || S > chunks ||
        (S - 1) * ((chunks + S - 1) / S) >= chunks || (((M + mparts - 1) / mparts + 15) & ~15) > 256 ||
        (mode == 1 && !part) || (mode != 1 && S != 1) || ((mode == 0 || mode == 2) && !y) ||
        (mode == 2 ? (I <= 0 || I % (TNB / 2) != 0) : (N <= 0 || N % TNB != 0)) ||
        (mode == 3 && (!part || !masks || !ids || n_masks < 1 || wwords < (N + 31) / 32)))
        return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    auto xx = (const uint16_t*)x;
    auto ww = (const uint16_t*)w;
    auto yy = (uint16_t*)y;
    auto pp = (float*)part;
    auto mk = (const uint32_t*)masks;
    auto mi = (const int32_t*)midx;
    switch (mode) {
        case 0: return launch_tgemm<TM_BF16>(xx, ww, yy, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 1: return launch_tgemm<TM_PART>(xx, ww, yy, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 2: return launch_tgemm<TM_SWIGLU>(xx, ww, yy, pp, M, 2 * I, K, S, mparts, I, st, nullptr, nullptr, 0, 0);
        case 3: {
            hipError_t e = launch_tgemm<TM_ARGMAX>(xx, ww, nullptr, pp, M, N, K, 1, mparts, 0, st, mk, mi, n_masks,
                                                   wwords);
            if (e != hipSuccess) return e;
            argmax_pairs_kernel<<<(M + kBlock / kWave - 1) / (kBlock / kWave), kBlock, 0, st>>>(
                (const float2*)part, 4 * (N / TNB), M, (int32_t*)ids);
            return hipGetLastError();
        }
        default: return hipErrorInvalidValue;
    }
}

// diagnostics: mode-1 partials with kernel parts switched off (probe & 3:
// PROBE above), 32-deep stages (probe & 16: 64-B image rows), a 2-stage
// ring (probe & 32)
int dmcp_tgemm_probe(int probe, const void* x, const void* w, void* part, int M, int N, int K, int S, int mparts,
                     void* stream) {
    const int kc = (probe & 16) && probe < 64 ? 32 : TKC_DEFAULT;  // 257+: KC 64
    const int chunks = K / kc;
    if (M <= 0 || !x || !w || !part || S < 1 || K % kc != 0 || S > chunks ||
        (S - 1) * ((chunks + S - 1) / S) >= chunks || N % TNB != 0 || (((M + mparts - 1) / mparts + 15) & ~15) > 256)
        return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    auto xx = (const uint16_t*)x;
    auto ww = (const uint16_t*)w;
    auto pp = (float*)part;
#define DMCP_TP(P, KC, CAP) \
    return launch_tgemm<TM_PART, P, KC, CAP>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0)
    switch (probe) {
        case 1: DMCP_TP(1, 64, 6);
        case 2: DMCP_TP(2, 64, 6);
        case 16: DMCP_TP(0, 32, 6);
        case 17: DMCP_TP(1, 32, 6);
        case 18: DMCP_TP(2, 32, 6);
        case 32: DMCP_TP(0, 64, 2);   // ring capped at 2 stages (1 in flight)
        case 34: DMCP_TP(2, 64, 2);
        // register-weight kernel: 64 + PROBE, 128 + D (weight stages ahead)
        case 64: return launch_tgemm_r<TM_PART>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 65: return launch_tgemm_r<TM_PART, 1>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 66: return launch_tgemm_r<TM_PART, 2>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 130: return launch_tgemm_r<TM_PART, 0, 2>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        // weight L2 prefetch 1 / 2 / 3 / 4 / 6 stages ahead (PF); 256: the plain kernel
        case 256: return launch_tgemm<TM_PART>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 257: return launch_tgemm<TM_PART, 0, 64, 6, 1>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 258: return launch_tgemm<TM_PART, 0, 64, 6, 2>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 259: return launch_tgemm<TM_PART, 0, 64, 6, 3>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 260: return launch_tgemm<TM_PART, 0, 64, 6, 4>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 262: return launch_tgemm<TM_PART, 0, 64, 6, 6>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        // the DMA ring alone (PROBE 2) with the weight prefetch 2 / 4 stages ahead
        case 274: return launch_tgemm<TM_PART, 2, 64, 6, 2>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 276: return launch_tgemm<TM_PART, 2, 64, 6, 4>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        case 129: return launch_tgemm_r<TM_PART, 0, 1>(xx, ww, nullptr, pp, M, N, K, S, mparts, 0, st, nullptr, nullptr, 0, 0);
        default: return hipErrorInvalidValue;
    }
#undef DMCP_TP
}

}  // extern "C"
