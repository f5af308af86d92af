// Prefill GEMMs on the MX-scaled fp8 matrix cores (gfx950 / MI355X, CDNA4):
//
//   Y[M, N] = (Aq[M, K] * 2^(As - 127)) . (Wq[N, K] * ws[N])^T      M in the thousands
//
// The batched prefill (dmcp.models.llm.LocalLM.prefill_batch: ~45 classes x
// ~560 own prompt tokens per admission, M ~ 25k rows) is compute-bound: its
// four projections per layer are ~93 % of its FLOPs.  hipBLASLt's bf16 GEMMs
// ran it at ~1.2 PFLOP/s; v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 operands
// retires twice the bf16 rate (MI355X_MICROARCH.md, matrix cores), and half
// the operand bytes per FLOP.  The operands:
//
//   * A (activations): MXFP8 -- e4m3 bytes with one power-of-two (E8M0) scale
//     per 32 consecutive K elements of a row.  The scale is an MFMA operand
//     (each lane's 32 k values ARE one scale block), so an activation needs
//     no whole-row statistics: the SwiGLU epilogue of the gate/up GEMM
//     quantises its own output tile (a row's 32 columns are the 32 lanes of a
//     half-wave) and the down projection consumes it directly;
//   * B (weights): e4m3 with one fp32 scale per output channel (quantised
//     once at load), applied in the epilogue; the MFMA's B scale is 1.
//
// Structure: 256 x 256 output tile per 256-thread block (one wave per SIMD),
// 4 waves as 2 (M) x 2 (N), each wave 4 x 4 tiles of 32 x 32 (256 accumulator
// registers).  At MX-fp8 rate the LDS is the tight resource: every k-step's
// fragment reads (16 KiB per wave) plus the DMA writes (32 KiB per block) must
// fit in the MFMA time -- 128 x 128 per wave reads 64 KiB per 64 k per block
// where 8 waves of 128 x 64 read 96 KiB (measured 1.2-1.8 PFLOP/s with 8
// waves, LDS-bound).  64-deep
// K stages (one MX MFMA k-step) staged by LDS-DMA (global_load_lds) into a
// 4-stage ring, 3 stages in flight, one counted vmcnt + raw s_barrier per
// stage (cdna_hip_programming.md §5, "Pipelining across barriers");
// [rows][4 x 16 B] LDS images with chunk j of row r in slot j ^ ((r >> 2) & 3)
// (the swizzle on the DMA's source address): the 16 lanes of a ds_read_b128
// pass cover all 64 banks.  The A scales of a stage ride the same ring
// (a 2-byte LDS-DMA per lane, landing as a dword), so the loop issues only one
// kind of load.
// Blocks are remapped so each XCD runs a contiguous range of tiles, grouped 8
// M tiles at a time (its 32 CUs share 8 A panels and 4 W tiles in L2).
//
// Fused epilogues (the accumulator lane holds column lane & 31 of 16 rows):
//   PM_BF16    y = bf16(acc * ws[n])
//   PM_RESID   resid += bf16(acc * ws[n])          (o / down projection)
//   PM_SWIGLU  act = silu(gate) * up -> MXFP8 act + E8M0 scales (gate / up
//              rows of the same 32 intermediate columns in one wave)
//   PM_QKV     RoPE on q / k (d and d + 32 of a 64-wide head in the same
//              lane), q written bf16, k / v appended to the KV cache
//              (bf16 or fp8) -- the rope_kv kernel folded in.
#include "dmcp_common.hpp"

namespace {

typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef int v4i_t __attribute__((ext_vector_type(4)));

// PG_PROBE (scripts/pgemm_probe.sh builds such variants; never the shipped
// library): 1 = the K loop issues no refill DMAs (stale stages: MFMA + LDS
// reads + barriers only), 2 = no per-stage barrier, 4 = block timeline
// stamps, 8 = the bf16 epilogue skips its global stores, 16 = nontemporal
// bf16 epilogue stores
#ifndef PG_PROBE
#define PG_PROBE 0
#endif
constexpr int PBM = 256, PBN = 256, PBK = 64, PST = 4, PTH = 256;
constexpr int PA_BYTES = PBM * PBK;                     // A image of a stage
constexpr int PB_BYTES = PBN * PBK;                     // W image
// A scales of the stage: a 2-byte LDS-DMA still writes a DWORD per lane (the
// value zero-extended; measured -- with 2-byte spacing each wave's upper
// lanes overwrote the next wave's slots and the last wave's the next stage's
// A image), so row r's 2 bytes sit at 4 r
constexpr int PS_BYTES = PBM * 4;
constexpr int PST_BYTES = PA_BYTES + PB_BYTES + PS_BYTES;
constexpr int PM_BF16 = 0, PM_RESID = 1, PM_SWIGLU = 2, PM_QKV = 3;
// BK = 128 (pgemm_kernel<..., 128>): 128-deep stages, [rows][8 x 16 B] images
// (full 128-B lines per DMA lane group, as tgemm.hip's measured 128-B rows),
// a two-slot ring, the stage's 4 A scale bytes per row as one 4-byte LDS-DMA
constexpr int PBK2 = 128;
constexpr int PA2_BYTES = PBM * PBK2, PB2_BYTES = PBN * PBK2, PS2_BYTES = PBM * 4;
constexpr int PST2_BYTES = PA2_BYTES + PB2_BYTES + PS2_BYTES;
template <int BK>
constexpr int pgemm_lds_bytes() { return BK == 128 ? 2 * PST2_BYTES : PST * PST_BYTES; }

struct PEpi {
    uint16_t* y;          // PM_BF16: out [M, N]; PM_RESID: resid [M, N] (in place)
    uint8_t* yq;          // PM_SWIGLU: act [M, I] e4m3
    uint8_t* ys;          // PM_SWIGLU: act scales [M, I / 32] E8M0
    int I;                // PM_SWIGLU: intermediate size (gate rows [0, I), up rows [I, 2I))
    // PM_QKV
    const int32_t* pos;
    const int32_t* slot;
    const float2* cos_sin;
    uint16_t* q_out;
    void* k_cache;
    void* v_cache;
    int Hq, Hkv, max_seq, max_pos, num_slots;
    int grp;              // M tiles per block-order group (dmcp_pgemm_set_group; 0 = 8)
};

// LDS-DMA of 16 / 4 / 2 bytes per lane (the size must be a literal)
template <int SIZE>
__device__ __forceinline__ void pglds(const void* src, void* lds_base) {
    auto g = (const __attribute__((address_space(1))) void*)src;
    auto l = (__attribute__((address_space(3))) void*)lds_base;
    if constexpr (SIZE == 16) __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
    else if constexpr (SIZE == 4) __builtin_amdgcn_global_load_lds(g, l, 4, 0, 0);
    else __builtin_amdgcn_global_load_lds(g, l, 2, 0, 0);
}

__device__ __forceinline__ int chunks_of(int K) { return K / PBK; }

__device__ __forceinline__ float psilu(float g) { return g / (1.f + __expf(-g)); }

// E8M0 exponent of a 32-element block of max |x| = amax: the smallest e with
// amax / 2^e <= 448 (e4m3's largest normal), clamped to the format
__device__ __forceinline__ int mx_exp(float amax) {
    if (!(amax > 0.f)) return 0;
    int e;
    frexpf(amax * (1.f / 448.f), &e);  // amax / 448 = f * 2^e, f in [0.5, 1)
    return e < -127 ? -127 : (e > 127 ? 127 : e);
}

// one byte of e4m3 (saturating)
__device__ __forceinline__ uint8_t to_fp8(float x) {
    return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(fp8_sat(x), 0.f, 0, false) & 0xffu);
}

// The operand layout of v_mfma_scale_f32_32x32x64_f8f6f4 with 8-bit
// operands (measured, scripts/mx_layout_probe.py): lane (r, h) = (l % 32,
// l / 32) holds row r (A) / column r (B); its bytes 0-15 are k 16 h .. 16 h
// + 15 and bytes 16-31 are k 32 + 16 h .. 32 + 16 h + 15; the E8M0 scale of
// lane (r, 0) scales the row's k block 0-31, that of lane (r, 1) block 32-63.
// In a stage row of 64 k bytes = 4 16-B chunks: lane half h reads chunks h
// and 2 + h, and the scale of block h.
#if (PG_PROBE & 4) != 0
// PG_PROBE & 4: per block (start, K loop done, epilogue done) s_memtime + the
// hardware id, for the block-timeline probe (scripts/pgemm_probe.py)
__device__ long long pg_stamps[65536][4];
#endif

// WV = 4: one wave per SIMD, 128 x 128 per wave (16 MFMAs, 9 LDS-DMA pieces
// per stage); WV = 8: two waves per SIMD, 128 x 64 per wave (8 MFMAs, 4-5
// pieces) -- one wave's MFMAs run while the other issues its DMAs.
// AR (128-deep stages only): the A operand's pieces through registers -- a
// global_load_dwordx4 per piece at the stage's start, its ds_write_b128 into
// the same swizzled image slot late in the stage -- so the LDS-DMA path
// carries only W (an LDS-DMA piece costs 100-185 issue cycles inside a busy
// phase, MI355X_MICROARCH.md; a register load a few)
template <int MODE, bool KV8, int WV, int BK = PBK, int AR = 0>
__global__ __launch_bounds__(WV * 64) __attribute__((amdgpu_waves_per_eu(WV / 4, WV / 4))) void pgemm_kernel(
    const uint8_t* __restrict__ aq, const uint8_t* __restrict__ as, const uint8_t* __restrict__ wq,
    const float* __restrict__ ws, int M, int N, int K, int mtiles, int ntiles, PEpi e) {
    constexpr int NU = WV == 4 ? 4 : 2;  // 32-column tiles per wave
    constexpr int WNW = WV / 2;          // waves along N
    constexpr int CPW = PBN / WNW;       // columns per wave
    constexpr int PPW = 16 / WV;         // 1-KiB LDS-DMA pieces per wave per operand per stage
    static_assert(BK == PBK || (BK == PBK2 && WV == 4), "128-deep stages: the 4-wave block only");
    __shared__ __attribute__((aligned(16))) uint8_t plds[pgemm_lds_bytes<BK>()];  // ONE LDS object
#if (PG_PROBE & 4) != 0
    const long long t_start = __builtin_amdgcn_s_memtime();
#endif

    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    const int wm = wv / WNW, wn = wv % WNW;
    const int l32 = lane & 31, hh = lane >> 5;
    const bool scl = WV == 4 || wv < 4;  // this wave fetches 64 rows' A scales per stage

    // block -> tile: XCD-contiguous ranges (bijective for any grid), then
    // 8 M tiles per group with N fastest inside the group's column
    const int nblk = mtiles * ntiles;
    const int b = blockIdx.x;
    const int xcd = b & 7, q8 = nblk >> 3, r8 = nblk & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int grp = e.grp > 0 ? e.grp : 8;
    const int per_group = grp * ntiles;
    const int gid = L / per_group;
    const int first = gid * grp;
    const int gsz = min(mtiles - first, grp);
    const int inn = L - gid * per_group;
    const int mt = first + inn % gsz, nt = inn / gsz;
    const int m0 = mt * PBM;

    // weight row of LDS image row r (SwiGLU: per wave CPW / 2 gate rows then
    // the up rows of the same intermediate columns)
    auto wrow = [&](int r) -> int {
        if constexpr (MODE == PM_SWIGLU) {
            const int w2 = r / CPW, t = (r % CPW) >= CPW / 2, i = r % (CPW / 2);
            return (t ? e.I : 0) + nt * 128 + w2 * (CPW / 2) + i;
        } else {
            return nt * PBN + r;
        }
    };

    // LDS-DMA sources: lane L of a 1-KiB piece fills image row base + L / 4,
    // slot L % 4 with logical 16-B chunk (L % 4) ^ ((row >> 2) & 3)
    const uint8_t* asrc[PPW];
    const uint8_t* wsrc[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int r = (wv * PPW + i) * 16 + (lane >> 2);
        const int ch = (lane & 3) ^ ((r >> 2) & 3);
        asrc[i] = aq + (size_t)min(m0 + r, M - 1) * K + ch * 16;
        wsrc[i] = wq + (size_t)wrow(r) * K + ch * 16;
    }
    // A scales: lane L of wave w fetches the stage's 2 bytes of row 64 w + L
    const int ksb = K >> 5;
    const uint8_t* ssrc = as + (size_t)min(m0 + (wv & 3) * 64 + lane, M - 1) * ksb;

    auto issue = [&](int c, int st) {
        uint8_t* base = plds + st * PST_BYTES;
#pragma unroll
        for (int i = 0; i < PPW; ++i) pglds<16>(asrc[i] + c * PBK, base + (wv * PPW + i) * 1024);
#pragma unroll
        for (int i = 0; i < PPW; ++i) pglds<16>(wsrc[i] + c * PBK, base + PA_BYTES + (wv * PPW + i) * 1024);
        if (scl) pglds<2>(ssrc + c * 2, base + PA_BYTES + PB_BYTES + (wv & 3) * 256);
    };

    f32x16_t acc[4][NU];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[t][u][i] = 0.f;

    // typed vector loads: they keep their TBAA tag, which is what lets the
    // waitcnt pass tell them from the LDS-DMA writes in flight (an untyped
    // LDS load -- e.g. a uint4 copied field by field -- gets a vmcnt(0) in
    // front of it, draining the ring every stage)
    auto frag = [&](const uint8_t* img, int r) -> v8i_t {
        const int sw = (r >> 2) & 3;
        const v4i_t lo = *reinterpret_cast<const v4i_t*>(img + r * PBK + (hh ^ sw) * 16);
        const v4i_t hi = *reinterpret_cast<const v4i_t*>(img + r * PBK + ((2 + hh) ^ sw) * 16);
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };

    // One K stage per step.  Stage c's first fragments (A tile 0 + its scale,
    // all of B) are already in registers, read at the end of step c - 1, so
    // the step opens on MFMAs: tile 0's 4 MFMAs (tile 1's reads behind the
    // first) with DMA pieces 0-3 of stage c + 3 threaded one per MFMA (an
    // LDS-DMA costs ~60 issue cycles, MI355X_MICROARCH.md, hidden behind a
    // 64-cycle MFMA), tile 1 with pieces 4-7 (tiles 2 and 3's reads behind its
    // first MFMA), tile 2 with piece 8; then the wait
    // for stage c + 1 (two newer stages in flight) and this wave's stage-c
    // reads, the raw barrier (stage c + 1 landed for every wave; no wave
    // reads slot c any more, so step c + 1 may refill it), stage c + 1's first
    // fragments into the other register set, and tile 3's MFMAs over their
    // latency.  sched_barrier pins the order.  The refill is unconditional
    // (past the last stage it re-reads it into the free slot, keeping the
    // block branch-free and the wait count constant).
    auto piece = [&](int i, int cc, int st) {
        if constexpr ((PG_PROBE & 1) != 0) return;
        uint8_t* base = plds + st * PST_BYTES;
        if (i < PPW) pglds<16>(asrc[i] + cc * PBK, base + (wv * PPW + i) * 1024);
        else if (i < 2 * PPW) pglds<16>(wsrc[i - PPW] + cc * PBK, base + PA_BYTES + (wv * PPW + i - PPW) * 1024);
        else if (scl) pglds<2>(ssrc + cc * 2, base + PA_BYTES + PB_BYTES + (wv & 3) * 256);
    };
    // LDS-DMA instructions of this wave per stage: the counted waits leave
    // two stages' worth in flight
    constexpr int GL_S = 2 * PPW + 1, GL_N = 2 * PPW;
    auto wait_stage = [&]() {  // stage c + 1 landed (this wave), stage c's reads done, then every wave
        if constexpr ((PG_PROBE & 1) != 0)
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else if (scl)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(GL_S * (PST - 2)) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(GL_N * (PST - 2)) : "memory");
        if constexpr ((PG_PROBE & 2) == 0) asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    struct Frags {
        v8i_t a0, b[NU];
        int s0;
    };
    auto stage_ptr = [&](int c) -> const uint8_t* { return plds + (c % PST) * PST_BYTES; };
    auto pre = [&](int c, Frags& F) {  // stage c: A tile 0 + scale, then B
        const uint8_t* A = stage_ptr(c);
        const int r = wm * 128 + l32;
        F.a0 = frag(A, r);
        F.s0 = A[PA_BYTES + PB_BYTES + r * 4 + hh];
#pragma unroll
        for (int u = 0; u < NU; ++u) F.b[u] = frag(A + PA_BYTES, wn * CPW + u * 32 + l32);
    };
    auto step = [&](int c, const Frags& F, Frags& G) {
        const uint8_t* A = stage_ptr(c);
        const uint8_t* S = A + PA_BYTES + PB_BYTES;
        const int cn = min(c + PST - 1, chunks_of(K) - 1), sn = (c + PST - 1) % PST;
        v8i_t af[4];
        int sa[4];
        auto aread = [&](int t) {
            const int r = wm * 128 + t * 32 + l32;
            af[t] = frag(A, r);
            sa[t] = S[r * 4 + hh];
        };
        auto mma = [&](int t, int u) {
            const v8i_t a = t == 0 ? F.a0 : af[t];
            const int sc = t == 0 ? F.s0 : sa[t];
            // C^T tile: A = 32 weight rows (scale 1), B = 32 activation rows
            // with their E8M0 block scales -> lane l32 holds activation row
            // t * 32 + l32, register i weight column (i & 3) + 8 (i >> 2) + 4 hh
            acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(F.b[u], a, acc[t][u], 0, 0, 0, 127, 0, sc);
        };
        // every read is issued right after an MFMA, ahead of its first use
        // (the waitcnt pass cannot count LDS reads past pending LDS-DMAs: each
        // use waits lgkmcnt(0), so nothing younger may be in flight then);
        // the DMA pieces one per MFMA from the first
        constexpr int NP = 2 * PPW + 1;
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int idx = t * NU + u;
                __builtin_amdgcn_sched_barrier(0);
                mma(t, u);
                __builtin_amdgcn_sched_barrier(0);
                if (idx == 0) aread(1);
                if (idx == NU) {
                    aread(2);
                    aread(3);
                }
                if (idx < NP) piece(idx, cn, sn);
            }
        __builtin_amdgcn_sched_barrier(0);
        wait_stage();
        pre(c + 1, G);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < NU; ++u) mma(3, u);
    };
    if constexpr (BK == PBK2) {
        // ---- 128-deep stages in a two-slot ring.  Step c computes stage c
        // (two MX k-steps of 64: 32 MFMAs per wave) while the 17 LDS-DMA
        // instructions of stage c + 1 go out one per MFMA into the other slot
        // (freed by the previous step's closing barrier).  Four MFMAs before
        // the end the wave waits for its own stage c + 1 pieces, the barrier
        // makes them every wave's (and retires every wave's stage-c reads),
        // and stage c + 1's first k-step fragments are read behind those
        // last MFMAs, so the next step opens on MFMAs.
        // Image rows of 128 B: chunk j of row r in slot j ^ ((r >> 1) & 7) --
        // the 16 lanes of each ds_read_b128 pass of the 32x32 operand layout
        // (rows {0-3,12-15,20-27} / {4-11,16-19,28-31}, one chunk) hit 16
        // distinct (row parity, slot) pairs: all 64 banks.
        constexpr int PP2 = PA2_BYTES / 1024 / WV;  // 1-KiB pieces per wave per operand per stage
        constexpr int NP2 = 2 * PP2 + 1;            // + the scale dword
        auto sw2 = [](int r) { return (r >> 1) & 7; };
        // 32-bit byte offsets of the pieces' sources (64-bit pointers for 16
        // pieces would hold 32 VGPRs through the loop)
        uint32_t a2[PP2], w2[PP2];
#pragma unroll
        for (int i = 0; i < PP2; ++i) {
            const int r = (wv * PP2 + i) * 8 + (lane >> 3);
            const int ch = (lane & 7) ^ sw2(r);
            a2[i] = (uint32_t)min(m0 + r, M - 1) * (uint32_t)K + ch * 16;
            w2[i] = (uint32_t)wrow(r) * (uint32_t)K + ch * 16;
        }
        const uint32_t s2 = (uint32_t)min(m0 + wv * 64 + lane, M - 1) * (uint32_t)ksb;  // 4 scale bytes per stage
        auto piece2 = [&](int i, int c2, int slot) {
            uint8_t* base = plds + slot * PST2_BYTES;
            const uint32_t kb = (uint32_t)c2 * PBK2;
            if (i < PP2) pglds<16>(aq + (a2[i] + kb), base + (wv * PP2 + i) * 1024);
            else if (i < 2 * PP2) pglds<16>(wq + (w2[i - PP2] + kb), base + PA2_BYTES + (wv * PP2 + i - PP2) * 1024);
            else pglds<4>(as + (s2 + (uint32_t)c2 * 4), base + PA2_BYTES + PB2_BYTES + wv * 256);
        };
        // AR: this stage's A pieces in flight in registers
        // The loads are inline asm, so the compiler's waitcnt pass (which
        // cannot count the LDS-DMAs in flight and would drain them all with a
        // vmcnt(0) before the first store) leaves the waits to astore: piece
        // i has PP2 - 1 - i younger A loads and the stage's W + scale DMAs
        // (NP2 - PP2) behind it.
        v4i_t areg[PP2];
        auto aload = [&](int i, int c2) {
            const uint8_t* src = aq + (a2[i] + (uint32_t)c2 * PBK2);
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(areg[i]) : "v"(src) : "memory");
        };
        auto astore = [&](int i, int slot) {
            switch (PP2 - 1 - i + NP2 - PP2) {  // vmcnt needs a literal
#define PG_VMW(n) case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
                PG_VMW(0) PG_VMW(1) PG_VMW(2) PG_VMW(3) PG_VMW(4) PG_VMW(5) PG_VMW(6) PG_VMW(7) PG_VMW(8)
                PG_VMW(9) PG_VMW(10) PG_VMW(11) PG_VMW(12) PG_VMW(13) PG_VMW(14) PG_VMW(15) PG_VMW(16)
#undef PG_VMW
                default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            *reinterpret_cast<v4i_t*>(plds + slot * PST2_BYTES + (wv * PP2 + i) * 1024 + lane * 16) = areg[i];
        };
        constexpr int AST0 = 8 * NU - 5 - PP2;  // MFMA index of the first A store (the last lands before the wait)
        auto frag2 = [&](const uint8_t* img, int r, int ks) -> v8i_t {
            const int sw = sw2(r);
            const v4i_t lo = *reinterpret_cast<const v4i_t*>(img + r * PBK2 + ((4 * ks + hh) ^ sw) * 16);
            const v4i_t hi = *reinterpret_cast<const v4i_t*>(img + r * PBK2 + ((4 * ks + 2 + hh) ^ sw) * 16);
            return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        };
        struct KF {
            v8i_t a[4], b[NU];
            int sc[4];
        };
        auto rd2 = [&](int c2, int ks, KF& F) {
            const uint8_t* A = plds + (c2 & 1) * PST2_BYTES;
            const uint8_t* S = A + PA2_BYTES + PB2_BYTES;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int r = wm * 128 + t * 32 + l32;
                F.a[t] = frag2(A, r, ks);
                F.sc[t] = S[r * 4 + 2 * ks + hh];
            }
#pragma unroll
            for (int u = 0; u < NU; ++u) F.b[u] = frag2(A + PA2_BYTES, wn * CPW + u * 32 + l32, ks);
        };
        const int chunks2 = K / PBK2;
        // branch-free (a guarded refill splits the step into blocks across which
        // the compiler moves the MFMAs, undoing the interleave): past the last
        // stage the refill re-reads that stage into the free slot and the next
        // k-step-0 read is of a slot nobody uses
        auto step2 = [&](int c, KF& F0, KF& F1) {  // F0: stage c, k-step 0 (read); F1: scratch -> next F0
            const int cn = min(c + 1, chunks2 - 1);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                KF& F = ks == 0 ? F0 : F1;
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int u = 0; u < NU; ++u) {
                        const int idx = ks * 4 * NU + t * NU + u;
                        __builtin_amdgcn_sched_barrier(0);
                        acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(F.b[u], F.a[t], acc[t][u], 0, 0, 0,
                                                                                    127, 0, F.sc[t]);
                        __builtin_amdgcn_sched_barrier(0);
                        if (idx == 0) rd2(c, 1, F1);  // k-step 1 of this stage, behind the first MFMA
                        if constexpr (AR != 0) {
                            if (idx < PP2) aload(idx, cn);
                            else if (idx < NP2) piece2(idx, cn, (c + 1) & 1);
                            if (idx >= AST0 && idx < AST0 + PP2) astore(idx - AST0, (c + 1) & 1);
                        } else if (idx < NP2) {
                            piece2(idx, cn, (c + 1) & 1);
                        }
                        if (idx == 8 * NU - 5) {  // four MFMAs before the end: stage c + 1 in, then its k-step 0
                            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                            asm volatile("s_barrier" ::: "memory");
                            __builtin_amdgcn_sched_barrier(0);
                            rd2(c + 1, 0, F0);
                        }
                    }
            }
        };
        // prologue: stage 0 in, its k-step 0 read
        if constexpr (AR != 0) {
#pragma unroll
            for (int i = 0; i < PP2; ++i) aload(i, 0);
            for (int i = PP2; i < NP2; ++i) piece2(i, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < PP2; ++i) astore(i, 0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else {
            for (int i = 0; i < NP2; ++i) piece2(i, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        KF Fa, Fb;
        rd2(0, 0, Fa);
        for (int c = 0; c < chunks2; ++c) step2(c, Fa, Fb);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
    const int chunks = chunks_of(K);
#pragma unroll
    for (int j = 0; j < PST - 1; ++j) issue(min(j, chunks - 1), j);
    // stage 0: landed for every wave, its first fragments read
    if constexpr ((PG_PROBE & 1) != 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (scl)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(GL_S * (PST - 2)) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(GL_N * (PST - 2)) : "memory");
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (WV == 8) {
        // two waves per SIMD: the partner wave hides this one's read latency,
        // so no second fragment set (it would not fit beside 128 accumulators
        // in a wave's 256 registers): each step waits for its stage, reads,
        // computes; the barrier at its top also retires every wave's reads of
        // the slot the step refills
        for (int c = 0; c < chunks; ++c) {
            if (c > 0) {
                if constexpr ((PG_PROBE & 1) != 0)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                else if (scl)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(GL_S * (PST - 2)) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(GL_N * (PST - 2)) : "memory");
                asm volatile("s_barrier" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
            }
            const uint8_t* A = stage_ptr(c);
            const uint8_t* S = A + PA_BYTES + PB_BYTES;
            const int cn = min(c + PST - 1, chunks - 1), sn = (c + PST - 1) % PST;
            v8i_t af[4], bf[NU];
            int sa[4];
            auto aread = [&](int t) {
                const int r = wm * 128 + t * 32 + l32;
                af[t] = frag(A, r);
                sa[t] = S[r * 4 + hh];
            };
            aread(0);
#pragma unroll
            for (int u = 0; u < NU; ++u) bf[u] = frag(A + PA_BYTES, wn * CPW + u * 32 + l32);
            constexpr int NP = 2 * PPW + 1;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const int idx = t * NU + u;
                    __builtin_amdgcn_sched_barrier(0);
                    acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bf[u], af[t], acc[t][u], 0, 0, 0, 127,
                                                                                0, sa[t]);
                    __builtin_amdgcn_sched_barrier(0);
                    if (idx == 0) aread(1);
                    if (idx == NU) {
                        aread(2);
                        aread(3);
                    }
                    if (idx < NP) piece(idx, cn, sn);
                }
        }
    } else {
        Frags F0, F1;
        pre(0, F0);
        // two steps per trip: the register sets swap roles by name, never by a
        // runtime index (cdna_hip_programming.md §5.4 rule 20)
        int c = 0;
        for (; c + 1 < chunks; c += 2) {
            step(c, F0, F1);
            step(c + 1, F1, F0);
        }
        if (c < chunks) step(c, F0, F1);
    }
    // the refills past the last stage land before the block's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }  // BK == PBK
#if (PG_PROBE & 4) != 0
    const long long t_loop = __builtin_amdgcn_s_memtime();
#endif

    // ---- epilogue, in registers.  Lane (l32, hh) holds row t * 32 + l32 of
    // the wave's tile and, per 32-column tile u, columns 8 j + 4 hh + q
    // (register 4 j + q): four 4-column groups.  A v_permlane32_swap of groups
    // (0, 1) and (2, 3) (cdna_hip_programming.md T21) leaves lanes 0-31 with
    // columns 0-7 and 16-23 and lanes 32-63 with 8-15 and 24-31: two 16-B
    // (bf16) or 8-B (fp8) stores per lane per tile, no LDS round trip.
    const int mw = m0 + wm * 128;  // first row of this wave's tile
    const int n0 = nt * PBN + wn * CPW;
    auto swap2 = [&](uint32_t& a, uint32_t& b) {  // lanes 32-63 of a <-> lanes 0-31 of b
        const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
        a = r[0];
        b = r[1];
    };
    // 16 values of a tile -> 4 packed bf16 groups, swapped into 2 x 16 B
    auto bf16_rows = [&](const float* v, uint4& lo, uint4& hi) {
        uint2 g[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) g[j] = pack4(v + 4 * j);
        swap2(g[0].x, g[1].x);
        swap2(g[0].y, g[1].y);
        swap2(g[2].x, g[3].x);
        swap2(g[2].y, g[3].y);
        lo = make_uint4(g[0].x, g[0].y, g[1].x, g[1].y);  // columns 8 hh .. + 7
        hi = make_uint4(g[2].x, g[2].y, g[3].x, g[3].y);  // columns 16 + 8 hh .. + 7
    };
    // 16 values -> 4 e4m3 groups (through bf16 when kv), swapped into 2 x 8 B
    auto fp8_rows = [&](const float* v, bool via_bf16, uint2& lo, uint2& hi) {
        uint32_t g[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) g[j] = via_bf16 ? pack_fp8x4_bf16r(v + 4 * j) : pack_fp8x4(v + 4 * j);
        swap2(g[0], g[1]);
        swap2(g[2], g[3]);
        lo = make_uint2(g[0], g[1]);
        hi = make_uint2(g[2], g[3]);
    };
    auto scales16 = [&](const float* base, float* sc) {  // sc[4 j + q] = base[8 j + 4 hh + q]
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 f = *reinterpret_cast<const float4*>(base + 8 * j + 4 * hh);
            sc[4 * j] = f.x;
            sc[4 * j + 1] = f.y;
            sc[4 * j + 2] = f.z;
            sc[4 * j + 3] = f.w;
        }
    };
    if constexpr (MODE == PM_BF16 || MODE == PM_RESID) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            float sc[16];
            scales16(ws + n0 + u * 32, sc);
            const int col = n0 + u * 32 + 8 * hh;
            uint4 r[4][2];
            if constexpr (MODE == PM_RESID) {  // the 8 residual chunks of this tile column in flight together
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint16_t* rp = e.y + (size_t)min(mw + t * 32 + l32, M - 1) * N + col;
                    r[t][0] = *reinterpret_cast<const uint4*>(rp);
                    r[t][1] = *reinterpret_cast<const uint4*>(rp + 16);
                }
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int m = mw + t * 32 + l32;
                float v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = acc[t][u][i] * sc[i];
                uint4 lo, hi;
                bf16_rows(v, lo, hi);
                if (m >= M) continue;
                uint16_t* dst = e.y + (size_t)m * N + col;
                if constexpr (MODE == PM_RESID) {
                    float a[8], b2[8];
                    unpack8(lo, a);
                    unpack8(r[t][0], b2);
#pragma unroll
                    for (int j = 0; j < 8; ++j) a[j] += b2[j];
                    lo = pack8(a);
                    unpack8(hi, a);
                    unpack8(r[t][1], b2);
#pragma unroll
                    for (int j = 0; j < 8; ++j) a[j] += b2[j];
                    hi = pack8(a);
                }
                *reinterpret_cast<uint4*>(dst) = lo;
                *reinterpret_cast<uint4*>(dst + 16) = hi;
            }
        }
    } else if constexpr (MODE == PM_SWIGLU) {
        // tiles u < NU / 2: gate columns j0 + 32 u .., tiles u + NU / 2: the
        // up columns of the same intermediates (the wrow interleave above)
        const int j0 = nt * 128 + wn * (CPW / 2);
        const int isb = e.I >> 5;
#pragma unroll
        for (int u = 0; u < NU / 2; ++u) {
            float sg[16], su[16];
            scales16(ws + j0 + u * 32, sg);
            scales16(ws + e.I + j0 + u * 32, su);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int m = mw + t * 32 + l32;
                float a[16];
                float amax = 0.f;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    // gate / up rounded to bf16 as the bf16 GEMM's outputs are
                    const float g = bf2f(f2bf(acc[t][u][i] * sg[i])), uu = bf2f(f2bf(acc[t][u + NU / 2][i] * su[i]));
                    a[i] = bf2f(f2bf(psilu(g) * uu));
                    amax = __builtin_fmaxf(amax, __builtin_fabsf(a[i]));
                }
                amax = half_swap_max(amax);  // the block's other 16 columns are in lane ^ 32
                const int ex = mx_exp(amax);
#pragma unroll
                for (int i = 0; i < 16; ++i) a[i] = ldexpf(a[i], -ex);
                uint2 lo, hi;
                fp8_rows(a, false, lo, hi);
                if (m >= M) continue;
                uint8_t* dst = e.yq + (size_t)m * e.I + j0 + u * 32 + 8 * hh;
                *reinterpret_cast<uint2*>(dst) = lo;
                *reinterpret_cast<uint2*>(dst + 16) = hi;
                if (hh == 0) e.ys[(size_t)m * isb + ((j0 + u * 32) >> 5)] = (uint8_t)(ex + 127);
            }
        }
    } else {  // PM_QKV: tiles 2 g, 2 g + 1 = d 0..31, 32..63 of head h0 + g
        const int h0 = n0 >> 6;
        const bool kv = h0 + NU / 2 - 1 >= e.Hq;  // some head of this wave goes to the caches
        int pos[4], sl[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int mc = min(mw + t * 32 + l32, M - 1);
            pos[t] = e.pos[mc];
            sl[t] = kv ? e.slot[mc] : -1;
        }
        float sc[NU][16];
#pragma unroll
        for (int u = 0; u < NU; ++u) scales16(ws + n0 + u * 32, sc[u]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int m = mw + t * 32 + l32;
            // (cos, sin) of d = 8 j + 4 hh + q: two float4 per group
            float cs_c[16], cs_s[16];
            const float4* tb = reinterpret_cast<const float4*>(
                e.cos_sin + (size_t)min(max(pos[t], 0), e.max_pos - 1) * 32);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 p0 = tb[(8 * j + 4 * hh) / 2], p1 = tb[(8 * j + 4 * hh) / 2 + 1];
                cs_c[4 * j] = p0.x; cs_s[4 * j] = p0.y; cs_c[4 * j + 1] = p0.z; cs_s[4 * j + 1] = p0.w;
                cs_c[4 * j + 2] = p1.x; cs_s[4 * j + 2] = p1.y; cs_c[4 * j + 3] = p1.z; cs_s[4 * j + 3] = p1.w;
            }
#pragma unroll
            for (int g = 0; g < NU / 2; ++g) {
                const int head = h0 + g;
                float lo[16], hi[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {  // the projection's bf16 outputs
                    lo[i] = bf2f(f2bf(acc[t][2 * g][i] * sc[2 * g][i]));
                    hi[i] = bf2f(f2bf(acc[t][2 * g + 1][i] * sc[2 * g + 1][i]));
                }
                if (head < e.Hq + e.Hkv) {  // rotate-half RoPE: d < 32: x c - x' s; d >= 32: x' c + x s
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const float a = lo[i], b = hi[i];
                        lo[i] = a * cs_c[i] - b * cs_s[i];
                        hi[i] = b * cs_c[i] + a * cs_s[i];
                    }
                }
                if (m >= M) continue;
                size_t ofs;  // element offset of d = 0 of this (row, head)
                void* base;
                bool to_cache = false;
                if (head < e.Hq) {
                    ofs = ((size_t)m * e.Hq + head) * 64;
                    base = e.q_out;
                } else {
                    const int pp = pos[t], sq = sl[t];
                    if (pp < 0 || pp >= e.max_seq || sq < 0 || sq >= e.num_slots) continue;
                    const bool isv = head >= e.Hq + e.Hkv;
                    const int kh = head - e.Hq - (isv ? e.Hkv : 0);
                    ofs = (((size_t)sq * e.Hkv + kh) * e.max_seq + pp) * 64;
                    base = isv ? e.v_cache : e.k_cache;
                    to_cache = true;
                }
                if (KV8 && to_cache) {
                    uint2 a0, a1, b0, b1;
                    fp8_rows(lo, true, a0, a1);
                    fp8_rows(hi, true, b0, b1);
                    uint8_t* d8 = static_cast<uint8_t*>(base) + ofs + 8 * hh;
                    *reinterpret_cast<uint2*>(d8) = a0;
                    *reinterpret_cast<uint2*>(d8 + 16) = a1;
                    *reinterpret_cast<uint2*>(d8 + 32) = b0;
                    *reinterpret_cast<uint2*>(d8 + 48) = b1;
                } else {
                    uint4 a0, a1, b0, b1;
                    bf16_rows(lo, a0, a1);
                    bf16_rows(hi, b0, b1);
                    uint16_t* d16 = static_cast<uint16_t*>(base) + ofs + 8 * hh;
                    *reinterpret_cast<uint4*>(d16) = a0;
                    *reinterpret_cast<uint4*>(d16 + 16) = a1;
                    *reinterpret_cast<uint4*>(d16 + 32) = b0;
                    *reinterpret_cast<uint4*>(d16 + 48) = b1;
                }
            }
        }
    }
#if (PG_PROBE & 4) != 0
    __syncthreads();
    if (tid == 0 && blockIdx.x < 65536) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        pg_stamps[blockIdx.x][0] = t_start;
        pg_stamps[blockIdx.x][1] = t_loop;
        pg_stamps[blockIdx.x][2] = __builtin_amdgcn_s_memtime();
        pg_stamps[blockIdx.x][3] = hw;
    }
#endif
}

// ---- decode: weight-streaming GEMM on MX fp8 (the wgemm.hip structure with
// e4m3 weights and MXFP8 activations: half the bytes of both operands per
// block -- the per-CU load path, not HBM, bounded the bf16 form)
//
//   C^T tile = W[n rows] . X[m rows]^T on v_mfma_scale_f32_32x32x64_f8f6f4:
//   A = 32 weight rows (scale 1: the per-row fp32 weight scale is applied
//   in the epilogue), B = 32 activation rows with their E8M0 block scales.
//   A lane holds activation row lane % 32 and 16 output columns
//   (i & 3) + 8 (i >> 2) + 4 (lane >> 5) of its tile.
//
// A block owns NB = 64 weight rows (SwiGLU: 32 gate + 32 up rows of the
// same intermediate columns) and all rows of its M part (MT x 128 rows,
// 4 waves x MT 32-row tiles), a K slice of K / S; LDS-DMA ring of 64-deep
// stages as pgemm_kernel.
constexpr int XM_PART = 1, XM_SWIGLU = 2;

template <int NB, int MT, int MODE, int ST>
__global__ __launch_bounds__(kBlock) void wmx_kernel(
    const uint8_t* __restrict__ xq, const uint8_t* __restrict__ xs, const uint8_t* __restrict__ wq,
    const float* __restrict__ ws, float* __restrict__ part, uint8_t* __restrict__ yq, uint8_t* __restrict__ ys,
    int M, int N, int K, int ks, int S, int ntiles, int mparts, int I) {
    constexpr int MR = MT * 128;                  // activation rows staged per block
    constexpr int NF = NB / 32;                   // weight tiles
    constexpr int W_BYTES = NB * PBK, X_BYTES = MR * PBK, XS_BYTES = 4 * kWave * 4;  // a dword per lane (see PS_BYTES)
    constexpr int STB = W_BYTES + X_BYTES + XS_BYTES;
    constexpr int WI = NB / 64;                   // 1-KiB weight pieces per wave per stage
    constexpr int XI = MR / 64;                   // activation pieces per wave
    constexpr int GL = WI + XI + 1;               // LDS-DMA instructions per wave per stage
    __shared__ __attribute__((aligned(16))) uint8_t lds[ST * STB];

    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    const int l32 = lane & 31, hh = lane >> 5;
    // block -> (weight tile, K slice, M part): the M parts of one (tile, slice)
    // share blockIdx % 8 (one XCD) and consecutive dispatch slots
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
    const int nt = u % ntiles, sl = u / ntiles;
    const int k0 = sl * ks;
    const int m_lo = mp * MR;

    auto wrow = [&](int r) -> int {
        if constexpr (MODE == XM_SWIGLU) return r < NB / 2 ? nt * (NB / 2) + r : I + nt * (NB / 2) + (r - NB / 2);
        else return nt * NB + r;
    };
    const uint8_t* wsrc[WI];
    const uint8_t* xsrc[XI];
#pragma unroll
    for (int i = 0; i < WI; ++i) {
        const int r = (wv * WI + i) * 16 + (lane >> 2);
        wsrc[i] = wq + (size_t)wrow(r) * K + k0 + (((lane & 3) ^ ((r >> 2) & 3)) * 16);
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {
        const int r = (wv * XI + i) * 16 + (lane >> 2);
        xsrc[i] = xq + (size_t)min(m_lo + r, M - 1) * K + k0 + (((lane & 3) ^ ((r >> 2) & 3)) * 16);
    }
    // activation scales: the stage's 2 bytes of each staged row; wave w, lane L
    // -> row w * (MR / 4) + L (MT = 1: lanes 32-63 repeat lanes 0-31)
    const int srow = wv * (MR / 4) + (MT == 2 ? lane : l32);
    const int ksb = K >> 5;
    const uint8_t* ssrc = xs + (size_t)min(m_lo + srow, M - 1) * ksb + (k0 >> 5);

    auto issue = [&](int c, int st) {
        uint8_t* base = lds + st * STB;
#pragma unroll
        for (int i = 0; i < WI; ++i) pglds<16>(wsrc[i] + c * PBK, base + (wv * WI + i) * 1024);
#pragma unroll
        for (int i = 0; i < XI; ++i) pglds<16>(xsrc[i] + c * PBK, base + W_BYTES + (wv * XI + i) * 1024);
        pglds<2>(ssrc + c * 2, base + W_BYTES + X_BYTES + wv * 256);
    };

    f32x16_t acc[NF][MT];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[f][t][i] = 0.f;

    auto frag = [&](const uint8_t* img, int r) -> v8i_t {
        const int sw = (r >> 2) & 3;
        const v4i_t lo = *reinterpret_cast<const v4i_t*>(img + r * PBK + (hh ^ sw) * 16);
        const v4i_t hi = *reinterpret_cast<const v4i_t*>(img + r * PBK + ((2 + hh) ^ sw) * 16);
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    auto compute = [&](int st) {
        const uint8_t* W = lds + st * STB;
        const uint8_t* X = W + W_BYTES;
        const uint8_t* SX = X + X_BYTES;
        v8i_t xf[MT];
        int sx[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const int r = wv * (MT * 32) + t * 32 + l32;  // staged activation row
            xf[t] = frag(X, r);
            // row r was fetched by wave r / (MR / 4), lane r % (MR / 4)
            sx[t] = SX[(r / (MR / 4)) * 256 + (r % (MR / 4)) * 4 + hh];
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const v8i_t wf = frag(W, f * 32 + l32);
#pragma unroll
            for (int t = 0; t < MT; ++t)
                acc[f][t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf, xf[t], acc[f][t], 0, 0, 0, 127, 0,
                                                                            sx[t]);
        }
    };

    const int chunks = ks / PBK;
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
        compute(c % ST);
    }

    // epilogue: lane holds activation row m, output columns (i & 3) + 8 (i >> 2) + 4 hh of tile f
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        const int m = m_lo + wv * (MT * 32) + t * 32 + l32;
        if constexpr (MODE == XM_PART) {
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int n = nt * NB + f * 32 + 8 * j + 4 * hh;
                    const float4 sc = *reinterpret_cast<const float4*>(ws + n);
                    if (m < M)
                        *reinterpret_cast<float4*>(part + ((size_t)sl * M + m) * N + n) =
                            make_float4(acc[f][t][4 * j] * sc.x, acc[f][t][4 * j + 1] * sc.y,
                                        acc[f][t][4 * j + 2] * sc.z, acc[f][t][4 * j + 3] * sc.w);
                }
        } else {  // XM_SWIGLU: tiles f = 0, 1 gate columns, f + 2 the up columns of the same intermediates
            const int isb = I >> 5;
#pragma unroll
            for (int f = 0; f < NF / 2; ++f) {
                float a[16];
                float amax = 0.f;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int jj = nt * (NB / 2) + f * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
                    const float g = bf2f(f2bf(acc[f][t][i] * ws[jj])), uu = bf2f(f2bf(acc[f + NF / 2][t][i] * ws[I + jj]));
                    a[i] = psilu(g) * uu;
                    amax = __builtin_fmaxf(amax, __builtin_fabsf(a[i]));
                }
                amax = half_swap_max(amax);  // the block's other 16 columns are in lane ^ 32
                const int ex = mx_exp(amax);
                const int jb = nt * (NB / 2) + f * 32;
#pragma unroll
                for (int i = 0; i < 16; ++i) a[i] = ldexpf(a[i], -ex);
                if (m < M) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        *reinterpret_cast<uint32_t*>(yq + (size_t)m * I + jb + 8 * j + 4 * hh) = pack_fp8x4(a + 4 * j);
                    if (hh == 0) ys[(size_t)m * isb + (jb >> 5)] = (uint8_t)(ex + 127);
                }
            }
        }
    }
}

// split-K reduction + residual add + RMSNorm, output MXFP8 (the next MX
// GEMM's activation): resid += bf16(sum_s part[s]); h = RMSNorm(resid) * w.
// One block per row, N % 2048 == 0, N <= 8192.
template <int VPT>
__global__ __launch_bounds__(kBlock) void reduce_resid_norm_mx_kernel(const float* __restrict__ part, int S,
                                                                      uint16_t* __restrict__ resid,
                                                                      const uint16_t* __restrict__ w,
                                                                      uint8_t* __restrict__ q, uint8_t* __restrict__ s,
                                                                      int M, int N, float eps) {
    const int m = blockIdx.x;
    uint4* rr = reinterpret_cast<uint4*>(resid + (size_t)m * N);
    const uint4* wr = reinterpret_cast<const uint4*>(w);
    float h[VPT][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        sum_slices8(part, S, M, m, N, idx, acc);
        float y[8], r[8];
        unpack8(pack8(acc), y);  // the GEMM output rounded to bf16, as F.linear's
        unpack8(rr[idx], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] += r[j];
        const uint4 packed = pack8(y);
        rr[idx] = packed;
        unpack8(packed, h[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += h[i][j] * h[i][j];
    }
    __shared__ float red[kBlock / kWave];
    ss = wave_sum(ss);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < kBlock / kWave; ++i) tot += red[i];
    const float inv = rsqrtf(tot / (float)N + eps);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        float g[8], o[8];
        unpack8(wr[idx], g);
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            o[j] = h[i][j] * inv * g[j];
            amax = __builtin_fmaxf(amax, __builtin_fabsf(o[j]));
        }
        amax = __builtin_fmaxf(amax, __shfl_xor(amax, 1, kWave));
        amax = __builtin_fmaxf(amax, __shfl_xor(amax, 2, kWave));
        const int ex = mx_exp(amax);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = ldexpf(o[j], -ex);
        reinterpret_cast<uint2*>(q + (size_t)m * N)[idx] = make_uint2(pack_fp8x4(o), pack_fp8x4(o + 4));
        if ((idx & 3) == 0) s[(size_t)m * (N >> 5) + (idx >> 2)] = (uint8_t)(ex + 127);
    }
}

// MXFP8 quantisation of bf16 rows: q[M, K] e4m3, s[M, K / 32] E8M0 (4 lanes
// per 32-block, 8 elements per lane)
__global__ __launch_bounds__(kBlock) void mx_quant_kernel(const uint16_t* __restrict__ x, uint8_t* __restrict__ q,
                                                          uint8_t* __restrict__ s, long n8) {
    for (long v = (long)blockIdx.x * kBlock + threadIdx.x; v < n8; v += (long)gridDim.x * kBlock) {
        float f[8];
        unpack8(reinterpret_cast<const uint4*>(x)[v], f);
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) amax = __builtin_fmaxf(amax, __builtin_fabsf(f[j]));
        amax = __builtin_fmaxf(amax, __shfl_xor(amax, 1, kWave));
        amax = __builtin_fmaxf(amax, __shfl_xor(amax, 2, kWave));
        const int ex = mx_exp(amax);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = ldexpf(f[j], -ex);
        reinterpret_cast<uint2*>(q)[v] = make_uint2(pack_fp8x4(f), pack_fp8x4(f + 4));
        if ((v & 3) == 0) s[v >> 2] = (uint8_t)(ex + 127);
    }
}

// resid += add (bf16, when add != null); h = RMSNorm(resid) * w; h -> MXFP8.
// One block per row (N <= 8192, N % 256 == 0).
template <int VPT>
__global__ __launch_bounds__(kBlock) void rmsnorm_mx_kernel(uint16_t* __restrict__ resid,
                                                            const uint16_t* __restrict__ add,
                                                            const uint16_t* __restrict__ w, uint8_t* __restrict__ q,
                                                            uint8_t* __restrict__ s, int N, float eps) {
    const int m = blockIdx.x;
    uint4* rr = reinterpret_cast<uint4*>(resid + (size_t)m * N);
    const uint4* ar = add ? reinterpret_cast<const uint4*>(add + (size_t)m * N) : nullptr;
    const uint4* wr = reinterpret_cast<const uint4*>(w);
    const int nvec = N >> 3;
    float h[VPT][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;
        if (idx < nvec) {
            unpack8(rr[idx], h[i]);
            if (ar) {
                float a[8];
                unpack8(ar[idx], a);
#pragma unroll
                for (int j = 0; j < 8; ++j) h[i][j] += a[j];
                const uint4 packed = pack8(h[i]);
                rr[idx] = packed;
                unpack8(packed, h[i]);
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
    for (int i = 0; i < kBlock / kWave; ++i) tot += red[i];
    const float inv = rsqrtf(tot / (float)N + eps);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * kBlock;  // nvec is a multiple of kBlock: every lane takes part
        float g[8], o[8];
        unpack8(wr[idx], g);
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            o[j] = h[i][j] * inv * g[j];
            amax = __builtin_fmaxf(amax, __builtin_fabsf(o[j]));
        }
        amax = __builtin_fmaxf(amax, __shfl_xor(amax, 1, kWave));
        amax = __builtin_fmaxf(amax, __shfl_xor(amax, 2, kWave));
        const int ex = mx_exp(amax);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = ldexpf(o[j], -ex);
        reinterpret_cast<uint2*>(q + (size_t)m * N)[idx] = make_uint2(pack_fp8x4(o), pack_fp8x4(o + 4));
        if ((idx & 3) == 0) s[(size_t)m * (N >> 5) + (idx >> 2)] = (uint8_t)(ex + 127);
    }
}

// one MX MFMA on given lane fragments: the operand-layout probe of the tests
__global__ void mx_probe_kernel(const v8i_t* a, const v8i_t* b, const int* sa, const int* sb, f32x16_t* c) {
    const int l = threadIdx.x;
    f32x16_t acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    c[l] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
}

int g_pgemm_waves = 4;  // dmcp_pgemm_set_waves: 4 (one wave per SIMD) or 8 (two)
// dmcp_pgemm_set_bk: K per LDS stage, 64 or 128 (4-wave block, K % 128 == 0).
// 128 by default: the Llama-shape layer at 24,576 rows 1,654 -> 1,564 us (down
// projection 405 -> 355 us; profiles/pgemm_bk128_r5.jsonl)
int g_pgemm_bk = 128;
int g_pgemm_group = 8;  // dmcp_pgemm_set_group: M tiles per block-order group
int g_pgemm_areg = 0;   // dmcp_pgemm_set_areg: A pieces through registers (128-deep stages)

template <int MODE, bool KV8>
hipError_t launch_pgemm(const void* aq, const void* as, const void* wq, const void* ws, int M, int N, int K,
                        const PEpi& e, void* stream) {
    const int mtiles = (M + PBM - 1) / PBM;
    const int ntiles = MODE == PM_SWIGLU ? e.I / 128 : N / PBN;
    PEpi e2 = e;
    e2.grp = g_pgemm_group;
    if (g_pgemm_bk == 128 && g_pgemm_waves == 4 && K % PBK2 == 0 && g_pgemm_areg)
        pgemm_kernel<MODE, KV8, 4, PBK2, 1><<<mtiles * ntiles, PTH, 0, (hipStream_t)stream>>>(
            (const uint8_t*)aq, (const uint8_t*)as, (const uint8_t*)wq, (const float*)ws, M, N, K, mtiles, ntiles, e2);
    else if (g_pgemm_bk == 128 && g_pgemm_waves == 4 && K % PBK2 == 0)
        pgemm_kernel<MODE, KV8, 4, PBK2><<<mtiles * ntiles, PTH, 0, (hipStream_t)stream>>>(
            (const uint8_t*)aq, (const uint8_t*)as, (const uint8_t*)wq, (const float*)ws, M, N, K, mtiles, ntiles, e2);
    else if (g_pgemm_waves == 8)
        pgemm_kernel<MODE, KV8, 8><<<mtiles * ntiles, 512, 0, (hipStream_t)stream>>>(
            (const uint8_t*)aq, (const uint8_t*)as, (const uint8_t*)wq, (const float*)ws, M, N, K, mtiles, ntiles, e2);
    else
        pgemm_kernel<MODE, KV8, 4><<<mtiles * ntiles, PTH, 0, (hipStream_t)stream>>>(
            (const uint8_t*)aq, (const uint8_t*)as, (const uint8_t*)wq, (const float*)ws, M, N, K, mtiles, ntiles, e2);
    return hipGetLastError();
}

bool pgemm_shape_ok(const void* aq, const void* as, const void* wq, const void* ws, int M, int N, int K) {
    return aq && as && wq && ws && M > 0 && K > 0 && K % PBK == 0 && N > 0 && N % PBN == 0;
}

}  // namespace

extern "C" {

// waves per block of the MX prefill GEMMs (4 or 8); returns the previous value
int dmcp_pgemm_set_waves(int w) {
    const int old = g_pgemm_waves;
    if (w == 4 || w == 8) g_pgemm_waves = w;
    return old;
}

// K per LDS stage of the MX prefill GEMMs (64 or 128); returns the previous value
int dmcp_pgemm_set_bk(int bk) {
    const int old = g_pgemm_bk;
    if (bk == 64 || bk == 128) g_pgemm_bk = bk;
    return old;
}

// A operand through registers instead of LDS-DMA (0 / 1, 128-deep stages); returns the previous value
int dmcp_pgemm_set_areg(int on) {
    const int old = g_pgemm_areg;
    if (on == 0 || on == 1) g_pgemm_areg = on;
    return old;
}

// M tiles per block-order group of the MX prefill GEMMs (1..64); returns the previous value
int dmcp_pgemm_set_group(int g) {
    const int old = g_pgemm_group;
    if (g >= 1 && g <= 64) g_pgemm_group = g;
    return old;
}

// mode 0: y[M, N] = bf16(A . W^T);  mode 1: y (= resid) += bf16(A . W^T).
// A: aq [M, K] e4m3 + as [M, K / 32] E8M0; W: wq [N, K] e4m3 + ws [N] fp32.
// Contract: K % 64 == 0, N % 256 == 0.
int dmcp_pgemm(const void* aq, const void* as, const void* wq, const void* ws, void* y, int M, int N, int K, int mode,
               void* stream) {
    if (M == 0) return 0;
    if (!pgemm_shape_ok(aq, as, wq, ws, M, N, K) || !y || (mode != 0 && mode != 1)) return hipErrorInvalidValue;
    PEpi e{};
    e.y = (uint16_t*)y;
    return mode == 0 ? launch_pgemm<PM_BF16, false>(aq, as, wq, ws, M, N, K, e, stream)
                     : launch_pgemm<PM_RESID, false>(aq, as, wq, ws, M, N, K, e, stream);
}

// act = silu(A . Wg^T) * (A . Wu^T) -> MXFP8 yq [M, I] + ys [M, I / 32];
// wq = [gate; up] [2I, K], ws [2I].  Contract: I % 128 == 0, K % 64 == 0.
int dmcp_pgemm_swiglu(const void* aq, const void* as, const void* wq, const void* ws, void* yq, void* ys, int M,
                      int I, int K, void* stream) {
    if (M == 0) return 0;
    if (!pgemm_shape_ok(aq, as, wq, ws, M, 256, K) || !yq || !ys || I <= 0 || I % 128 != 0)
        return hipErrorInvalidValue;
    PEpi e{};
    e.yq = (uint8_t*)yq;
    e.ys = (uint8_t*)ys;
    e.I = I;
    return launch_pgemm<PM_SWIGLU, false>(aq, as, wq, ws, M, 2 * I, K, e, stream);
}

// qkv = A . W^T (W [(Hq + 2 Hkv) 64, K]); RoPE on q / k; q_out [M, Hq, 64]
// bf16; k / v appended at (slot[m], :, pos[m], :) of the caches (kv8: e4m3).
// Contract: head dim 64, (Hq + 2 Hkv) % 4 == 0, K % 64 == 0.
int dmcp_pgemm_qkv(const void* aq, const void* as, const void* wq, const void* ws, const void* pos, const void* slot,
                   const void* cos_sin, void* q_out, void* k_cache, void* v_cache, int M, int K, int Hq, int Hkv,
                   int max_seq, int max_pos, int num_slots, int kv8, void* stream) {
    if (M == 0) return 0;
    const int N = (Hq + 2 * Hkv) * 64;
    if (!pgemm_shape_ok(aq, as, wq, ws, M, N, K) || !pos || !slot || !cos_sin || !q_out || !k_cache || !v_cache ||
        max_pos <= 0 || Hq <= 0 || Hkv <= 0)
        return hipErrorInvalidValue;
    PEpi e{};
    e.pos = (const int32_t*)pos;
    e.slot = (const int32_t*)slot;
    e.cos_sin = (const float2*)cos_sin;
    e.q_out = (uint16_t*)q_out;
    e.k_cache = k_cache;
    e.v_cache = v_cache;
    e.Hq = Hq;
    e.Hkv = Hkv;
    e.max_seq = max_seq;
    e.max_pos = max_pos;
    e.num_slots = num_slots;
    return kv8 ? launch_pgemm<PM_QKV, true>(aq, as, wq, ws, M, N, K, e, stream)
               : launch_pgemm<PM_QKV, false>(aq, as, wq, ws, M, N, K, e, stream);
}

// bf16 x [M, K] -> MXFP8 q [M, K] + s [M, K / 32]  (K % 32 == 0)
int dmcp_mx_quant(const void* x, void* q, void* s, int M, int K, void* stream) {
    if (M == 0) return 0;
    if (!x || !q || !s || K % 32 != 0) return hipErrorInvalidValue;
    const long n8 = (long)M * K / 8;
    const int grid = (int)std::min<long>((n8 + kBlock - 1) / kBlock, 8192);
    mx_quant_kernel<<<grid, kBlock, 0, (hipStream_t)stream>>>((const uint16_t*)x, (uint8_t*)q, (uint8_t*)s, n8);
    return hipGetLastError();
}

// resid += add (optional); RMSNorm(resid) * w -> MXFP8  (N % 2048 == 0, N <= 8192)
int dmcp_rmsnorm_mx(void* resid, const void* add, const void* w, void* q, void* s, int M, int N, float eps,
                    void* stream) {
    if (M == 0) return 0;
    if (!resid || !w || !q || !s || N % (8 * kBlock) != 0 || N > 4 * 8 * kBlock) return hipErrorInvalidValue;
    const int vpt = N / (8 * kBlock);
    auto st = (hipStream_t)stream;
    auto rr = (uint16_t*)resid;
    auto aa = (const uint16_t*)add;
    auto ww = (const uint16_t*)w;
    auto qq = (uint8_t*)q;
    auto ss = (uint8_t*)s;
    if (vpt == 1) rmsnorm_mx_kernel<1><<<M, kBlock, 0, st>>>(rr, aa, ww, qq, ss, N, eps);
    else if (vpt == 2) rmsnorm_mx_kernel<2><<<M, kBlock, 0, st>>>(rr, aa, ww, qq, ss, N, eps);
    else if (vpt == 3) rmsnorm_mx_kernel<3><<<M, kBlock, 0, st>>>(rr, aa, ww, qq, ss, N, eps);
    else rmsnorm_mx_kernel<4><<<M, kBlock, 0, st>>>(rr, aa, ww, qq, ss, N, eps);
    return hipGetLastError();
}

// Decode GEMMs on MX fp8 (contract checked by dmcp/ops/hip.py, guarded here):
// x MXFP8 [M, K] (+ [M, K / 32] scales), w e4m3 [N, K] + fp32 scales [N];
// M <= 1024, K % (64 S) == 0, rows / part <= 256.
//   mode 1: part[S, M, N] fp32 partials (N % 64 == 0)
//   mode 2: SwiGLU -> MXFP8 yq [M, I] + ys [M, I / 32]  (w = [gate; up] [2I, K], I % 32 == 0, S == 1)
int dmcp_wgemm_mx(const void* xq, const void* xs, const void* wq, const void* ws, void* part, void* yq, void* ys,
                  int M, int N, int K, int S, int mparts, int mode, int I, void* stream) {
    if (M <= 0) return 0;
    const int mrows = (M + mparts - 1) / mparts;
    if (!xq || !xs || !wq || !ws || M > 1024 || S < 1 || mparts < 1 || K % (PBK * S) != 0 || mrows > 256 ||
        (mode == 1 && (!part || N % 64 != 0)) || (mode == 2 && (!yq || !ys || S != 1 || I <= 0 || I % 32 != 0)) ||
        (mode != 1 && mode != 2))
        return hipErrorInvalidValue;
    auto st = (hipStream_t)stream;
    auto xx = (const uint8_t*)xq;
    auto xsc = (const uint8_t*)xs;
    auto ww = (const uint8_t*)wq;
    auto wsc = (const float*)ws;
    const int ks = K / S;
    const int mt = mrows > 128 ? 2 : 1;
    // the kernel stages MT x 128 rows per part from row mp * MT * 128
    if (mparts * mt * 128 < M) return hipErrorInvalidValue;
    if (mode == 1) {
        const int ntiles = N / 64;
        const dim3 grid((unsigned)(ntiles * S * mparts));
        if (mt == 2)
            wmx_kernel<64, 2, XM_PART, 4><<<grid, kBlock, 0, st>>>(xx, xsc, ww, wsc, (float*)part, nullptr, nullptr,
                                                                   M, N, K, ks, S, ntiles, mparts, 0);
        else
            wmx_kernel<64, 1, XM_PART, 4><<<grid, kBlock, 0, st>>>(xx, xsc, ww, wsc, (float*)part, nullptr, nullptr,
                                                                   M, N, K, ks, S, ntiles, mparts, 0);
    } else {
        // 64 gate + 64 up rows per block (half the activation re-staging of
        // 32 + 32: at 320 rows the staged activation bytes were twice the
        // weight bytes) once I / 64 tiles x parts fill the chip; else 32 + 32
        const bool wide = I % 64 == 0 && (I / 64) * mparts >= 256;
        const int ntiles = wide ? I / 64 : I / 32;
        const dim3 grid((unsigned)(ntiles * mparts));
#define DMCP_WMX_SW(NB, MT)                                                                                   \
    wmx_kernel<NB, MT, XM_SWIGLU, 4><<<grid, kBlock, 0, st>>>(xx, xsc, ww, wsc, nullptr, (uint8_t*)yq,        \
                                                              (uint8_t*)ys, M, 2 * I, K, K, 1, ntiles, mparts, I)
        if (wide) {
            if (mt == 2) DMCP_WMX_SW(128, 2);
            else DMCP_WMX_SW(128, 1);
        } else {
            if (mt == 2) DMCP_WMX_SW(64, 2);
            else DMCP_WMX_SW(64, 1);
        }
#undef DMCP_WMX_SW
    }
    return hipGetLastError();
}

// resid += bf16(sum of the S partials); RMSNorm(resid) * w -> MXFP8 q / s
int dmcp_reduce_resid_norm_mx(const void* part, int S, void* resid, const void* w, void* q, void* s, int M, int N,
                              float eps, void* stream) {
    if (M <= 0) return 0;
    if (!part || S < 1 || !resid || !w || !q || !s || N % (8 * kBlock) != 0 || N > 4 * 8 * kBlock)
        return hipErrorInvalidValue;
    const int vpt = N / (8 * kBlock);
    auto st = (hipStream_t)stream;
    auto pp = (const float*)part;
    auto rr = (uint16_t*)resid;
    auto ww = (const uint16_t*)w;
    auto qq = (uint8_t*)q;
    auto ss = (uint8_t*)s;
    if (vpt == 1) reduce_resid_norm_mx_kernel<1><<<M, kBlock, 0, st>>>(pp, S, rr, ww, qq, ss, M, N, eps);
    else if (vpt == 2) reduce_resid_norm_mx_kernel<2><<<M, kBlock, 0, st>>>(pp, S, rr, ww, qq, ss, M, N, eps);
    else if (vpt == 3) reduce_resid_norm_mx_kernel<3><<<M, kBlock, 0, st>>>(pp, S, rr, ww, qq, ss, M, N, eps);
    else reduce_resid_norm_mx_kernel<4><<<M, kBlock, 0, st>>>(pp, S, rr, ww, qq, ss, M, N, eps);
    return hipGetLastError();
}

#if (PG_PROBE & 4) != 0
int dmcp_pg_stamps(void* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(pg_stamps), (size_t)n * 4 * sizeof(long long), 0,
                               hipMemcpyDeviceToHost);
}
#endif

int dmcp_mx_probe(const void* a, const void* b, const void* sa, const void* sb, void* c, void* stream) {
    mx_probe_kernel<<<1, kWave, 0, (hipStream_t)stream>>>((const v8i_t*)a, (const v8i_t*)b, (const int*)sa,
                                                          (const int*)sb, (f32x16_t*)c);
    return hipGetLastError();
}

}  // extern "C"
