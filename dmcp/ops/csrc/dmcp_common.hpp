// Shared device helpers of the dmcp gfx950 kernels (dmcp_kernels.hip,
// fused_gemm.hip): bf16 <-> fp32 packing, wave reductions, MFMA operand
// types.  Header-only, everything in an anonymous namespace per TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace {

constexpr int kBlock = 256;
constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(uint16_t v) {
    return __uint_as_float(((uint32_t)v) << 16);
}

typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
typedef float f32x2v_t __attribute__((ext_vector_type(2)));

// round-to-nearest-even fp32 -> bf16 (NaN kept quiet): one v_cvt_pk_bf16_f32
// (the bit-twiddling form compiled to a NaN branch per value -- 256 divergent
// branches in a GEMM epilogue)
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// two floats -> packed bf16 pair (lo = a), one instruction
__device__ __forceinline__ uint32_t f2bf2(float a, float b) {
    const f32x2v_t v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v_t));
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
    f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
    uint4 v;
    v.x = f2bf2(f[0], f[1]);
    v.y = f2bf2(f[2], f[3]);
    v.z = f2bf2(f[4], f[5]);
    v.w = f2bf2(f[6], f[7]);
    return v;
}

__device__ __forceinline__ void unpack4(const uint2& v, float* f) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
}

__device__ __forceinline__ uint2 pack4(const float* f) {
    uint2 v;
    v.x = f2bf2(f[0], f[1]);
    v.y = f2bf2(f[2], f[3]);
    return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
    return v;
}

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short v4i16_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8_t as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8_t, v); }

// x of this lane and of lane ^ 32, through v_permlane32_swap (a VALU lane
// swap; __shfl_xor(x, 32) goes through an LDS ds_bpermute round trip).
// After the swap one result holds this lane's value and the other the
// partner half's, so symmetric ops (max, +) need not know which is which.
__device__ __forceinline__ float half_swap_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __builtin_fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ float half_swap_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ---- FP8 KV cache (OCP e4m3fn, gfx950's native fp8): unit scale, values
// saturated to +-448 on the way in (the hardware conversion does not clamp).
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float fp8_sat(float x) { return __builtin_fminf(__builtin_fmaxf(x, -448.f), 448.f); }

// 4 floats -> 4 e4m3 bytes (v_cvt_pk_fp8_f32 x2)
__device__ __forceinline__ uint32_t pack_fp8x4(const float* f) {
    const uint32_t lo = __builtin_amdgcn_cvt_pk_fp8_f32(fp8_sat(f[0]), fp8_sat(f[1]), 0, false);
    return __builtin_amdgcn_cvt_pk_fp8_f32(fp8_sat(f[2]), fp8_sat(f[3]), lo, true);
}

// 4 floats rounded to bf16 first, then e4m3: the bytes of a K-cache append
// (the reference rotates the bf16 projection in fp32, rounds to bf16, then
// encodes; a direct fp32 -> e4m3 differs by one e4m3 step where the bf16
// rounding lands on an e4m3 midpoint)
__device__ __forceinline__ uint32_t pack_fp8x4_bf16r(const float* f) {
    float r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = bf2f(f2bf(f[i]));
    return pack_fp8x4(r);
}

// 8 bf16 (uint4) -> 8 e4m3 bytes (uint2)
__device__ __forceinline__ uint2 bf16x8_to_fp8x8(const uint4& v) {
    float f[8];
    unpack8(v, f);
    return make_uint2(pack_fp8x4(f), pack_fp8x4(f + 4));
}

// 4 e4m3 bytes -> 4 bf16 (uint2): v_cvt_scalef32_pk_bf16_fp8 x2 (scale 1)
__device__ __forceinline__ uint2 fp8x4_to_bf16x4(uint32_t v) {
    return make_uint2(__builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v, 1.f, false)),
                      __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v, 1.f, true)));
}

// 8 e4m3 bytes -> 8 bf16 (uint4)
__device__ __forceinline__ uint4 fp8x8_to_bf16x8(const uint2& v) {
    const uint2 a = fp8x4_to_bf16x4(v.x), b = fp8x4_to_bf16x4(v.y);
    return make_uint4(a.x, a.y, b.x, b.y);
}

// byte address of element `off` of a bf16 or fp8 (KV8) cache
template <bool KV8>
__device__ __forceinline__ const void* kv_ptr(const void* base, size_t off) {
    return static_cast<const uint8_t*>(base) + off * (KV8 ? 1 : 2);
}

// h[0..7] += sum over split-K slices s < S of part[(s * M + m) * N + 8 idx ..
// + 7] (fp32 partials), RSU slices' loads in flight at once: a plain loop
// over s waited for each slice before issuing the next (S serial round trips
// per reduction).  Branch-free (a guarded add let the loads sink to their
// uses); the clamped surplus loads repeat the last slice with weight 0.
template <int RSU = 4>
__device__ __forceinline__ void sum_slices8(const float* __restrict__ part, int S, int M, int m, int N, int idx,
                                            float (&h)[8]) {
    for (int s0 = 0; s0 < S; s0 += RSU) {
        float4 a[RSU], b[RSU];
#pragma unroll
        for (int j = 0; j < RSU; ++j) {
            const float4* pp = reinterpret_cast<const float4*>(part + ((size_t)min(s0 + j, S - 1) * M + m) * N);
            a[j] = pp[2 * idx];
            b[j] = pp[2 * idx + 1];
        }
#pragma unroll
        for (int j = 0; j < RSU; ++j) {
            const float u = s0 + j < S ? 1.f : 0.f;
            h[0] = fmaf(u, a[j].x, h[0]); h[1] = fmaf(u, a[j].y, h[1]);
            h[2] = fmaf(u, a[j].z, h[2]); h[3] = fmaf(u, a[j].w, h[3]);
            h[4] = fmaf(u, b[j].x, h[4]); h[5] = fmaf(u, b[j].y, h[5]);
            h[6] = fmaf(u, b[j].z, h[6]); h[7] = fmaf(u, b[j].w, h[7]);
        }
    }
}

// The LM head's per-row selection from per-tile (max, id) pairs (wgemm.hip /
// tgemm.hip MODE_ARGMAX write best[tile * M + row]): the highest value, the
// lowest id among ties; 0 when the mask allowed nothing (as masked_argmax).
// One wave per row; each lane keeps 8 pairs' loads in flight (a plain
// strided loop waited for every load: ~30 serial round trips per row at
// 128,256 ids).  A clamped duplicate of the last pair never changes the result.
__global__ __launch_bounds__(kBlock) void argmax_pairs_kernel(const float2* __restrict__ best, int ntiles, int M,
                                                              int32_t* __restrict__ ids) {
    constexpr int U = 8;
    const int lane = threadIdx.x & (kWave - 1);
    const int m = blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
    if (m >= M) return;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int t0 = lane; t0 < ntiles; t0 += U * kWave) {
        float2 p[U];
#pragma unroll
        for (int j = 0; j < U; ++j) p[j] = best[(size_t)min(t0 + j * kWave, ntiles - 1) * M + m];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int pi = __float_as_int(p[j].y);
            if (p[j].x > bv || (p[j].x == bv && pi < bi)) { bv = p[j].x; bi = pi; }
        }
    }
#pragma unroll
    for (int msk = 32; msk >= 1; msk >>= 1) {
        const float ob = __shfl_xor(bv, msk, kWave);
        const int oi = __shfl_xor(bi, msk, kWave);
        if (ob > bv || (ob == bv && oi < bi)) { bv = ob; bi = oi; }
    }
    if (lane == 0) ids[m] = bi == 0x7fffffff ? 0 : bi;
}

}  // namespace
