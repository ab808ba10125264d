// Training-side GEMMs for the narrow projections (qkv: N 1152, o: N 896) of the
// full-sequence pass, where hipBLASLt's best solutions for M = 17408, K = 896 run at
// 0.4-0.8 PFLOP/s (profiles/r3_gemm_eff.log, profiles/r4_tgemm_pipe.log):
//
//   gemm_nt:  C[M, N] = A[M, K] · B[N, K]^T (+ bias[N])   forward / input gradient (SWH_TGEMM=all)
//   gemm_tn:  part[s] = dY[tokens of s]^T X, folded        weight gradient (default)
//
// bf16 in / out, fp32 accumulation.  gemm_nt:
// 128 x 128 output tiles, 4 waves (2 x 2, 64 x 64 each on v_mfma_f32_32x32x16_bf16),
// 64-wide K steps staged by LDS-DMA (global_load_lds, 16 B per lane) into a double
// buffer of 64 KB (two workgroups per CU).  The LDS image is lane-linear; the bank
// swizzle is applied on the SOURCE side (a row's 16-B chunk c lands at position
// c ^ ((row >> 1) & 7)) and undone on the read, which makes every ds_read_b128 of
// the 32 x 32 operand conflict-free (rows 2r and 2r+1 share a 256-B bank row).
// Tiles are mapped XCD-contiguous (bijective remap), so the N tiles of one M row
// block run on one XCD and read their A rows from its L2.  The K order of the sum
// is fixed (k-step by k-step, 16 k per MFMA): a row's result does not depend on
// where the row sits in the batch.
#include "common.hpp"

namespace swh {
namespace {

constexpr int kGT = 128;   // tile rows / columns
constexpr int kGK = 64;    // K granule of the shapes served (the K step is BK = 32 or 64)
constexpr int kGThreads = 256;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8g as_bf(const uint4 &v) { return __builtin_bit_cast(bf16x8g, v); }

// LDS reads as inline asm, so that the next k-step's fragments are requested before the
// current k-step's MFMAs (the compiler's own reads waited for each other); the caller
// waits (lgkmcnt) before using the data.
typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2g __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t lds_off(const unsigned char *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char *)p;
}
__device__ __forceinline__ uint4 lds_rd128(uint32_t a) {
    u32x4g v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return uint4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ uint2 lds_rd_tr16(uint32_t a) {
    u32x2g v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
    return uint2{v.x, v.y};
}
__device__ __forceinline__ void lgkm_wait0() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs behind the wait (they touch no memory)
}

// byte offset of 16-B chunk c of tile row r in the swizzled [128][BK] image: rows of
// 2 BK bytes, 256 / (2 BK) rows per 256-B bank row; chunk c sits at c ^ (bank row % chunks)
template <int BK>
__device__ __forceinline__ int gsw(int r, int c) {
    constexpr int CPR = BK / 8, SH = (BK == 64) ? 1 : 2;
    return r * (BK * 2) + ((c ^ ((r >> SH) & (CPR - 1))) << 4);
}

// The K loop over the two LDS stages: issue the next stage, compute this one, drain,
// barrier.  (Deeper pipelines measured no faster: 3-4 stages of 32- or 64-wide K steps
// with counted vmcnt waits across raw barriers)
template <int NS, int LPS, typename Stage, typename Compute>
__device__ __forceinline__ void gemm_kloop(int nk, Stage stage, Compute compute) {
    static_assert(NS == 2, "two stages");
    if (nk <= 0) return;
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ks = 0; ks < nk; ++ks) {
        if (ks + 1 < nk) stage((ks + 1) & 1, ks + 1);
        compute(ks & 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

template <bool BIAS, int NS, int BK>
__global__ __launch_bounds__(kGThreads) void gemm_nt_kernel(const uint16_t *__restrict__ A,
                                                            const uint16_t *__restrict__ B,
                                                            const uint16_t *__restrict__ bias, uint16_t *__restrict__ C,
                                                            int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gl[];  // [NS buffers][A | B]
    constexpr int SB = kGT * BK * 2, JL = BK / 16, CPR = BK / 8, RPI = 512 / BK, SH = (BK == 64) ? 1 : 2;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // XCD-contiguous tile order: workgroup ids land on XCD id % 8 round robin
    const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
    const int t = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
    const int ntn = N / kGT;
    const int m0 = (t / ntn) * kGT, n0 = (t % ntn) * kGT;
    const int nk = K / BK;

    // staging: wave w's load j fills image bytes [(4 j + w) KB, +1 KB) = RPI rows from
    // RPI (4 j + w), lane l -> row RPI (4 j + w) + l / CPR, position l % CPR, holding
    // source chunk (l % CPR) ^ swz
    const uint16_t *asrc[4], *bsrc[4];  // JL <= 4 used (a dependent extent breaks the host pass)
#pragma unroll
    for (int j = 0; j < JL; ++j) {
        const int row = RPI * (4 * j + wid) + lane / CPR;
        const int c = (lane % CPR) ^ ((row >> SH) & (CPR - 1));
        asrc[j] = A + (int64_t)min(m0 + row, M - 1) * lda + c * 8;
        bsrc[j] = B + (int64_t)(n0 + row) * ldb + c * 8;
    }
    auto stage = [=](int buf, int ks) {
        unsigned char *ai = gl + buf * 2 * SB, *bi = ai + SB;
        const int k0 = ks * BK;
#pragma unroll
        for (int j = 0; j < JL; ++j) {
            __builtin_amdgcn_global_load_lds(asrc[j] + k0, (__attribute__((address_space(3))) void *)(ai + (4 * j + wid) * 1024),
                                             16, 0, 0);
            __builtin_amdgcn_global_load_lds(bsrc[j] + k0, (__attribute__((address_space(3))) void *)(bi + (4 * j + wid) * 1024),
                                             16, 0, 0);
        }
    };

    const int wm = wid >> 1, wn = wid & 1, r32 = lane & 31, h = lane >> 5;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const uint32_t g0 = lds_off(gl);
    gemm_kloop<NS, 2 * JL>(nk, stage, [&](int cur) {
        const uint32_t ai = g0 + cur * 2 * SB, bi = ai + SB;
        uint4 a[2][2], b[2][2];  // [k-step parity][block]: the next k-step's fragments load under the MFMAs
        auto rd = [&](int kk) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                a[kk & 1][i] = lds_rd128(ai + gsw<BK>(wm * 64 + i * 32 + r32, 2 * kk + h));
                b[kk & 1][i] = lds_rd128(bi + gsw<BK>(wn * 64 + i * 32 + r32, 2 * kk + h));
            }
        };
        rd(0);
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            lgkm_wait0();
            if (kk + 1 < BK / 16) rd(kk + 1);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(a[kk & 1][i]), as_bf(b[kk & 1][j]),
                                                                        acc[i][j], 0, 0, 0);
        }
    });

    // epilogue: the wave's 64 x 64 bf16 tile through LDS (row pitch 72 elements), then
    // 16-B row stores: lane l -> row l / 8 + 8 it, columns 8 (l % 8) .. +7
    constexpr int P = 64 + 8;
    uint16_t *ct = reinterpret_cast<uint16_t *>(gl) + wid * 64 * P;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = wn * 64 + j * 32 + r32;
        const float bz = BIAS ? bf16_bits_to_f32(bias[n0 + col]) : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                ct[row * P + j * 32 + r32] = f32_to_bf16_bits(acc[i][j][e] + bz);
            }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own LDS writes done (wave-private region)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int row = it * 8 + (lane >> 3), c8 = (lane & 7) * 8;
        const uint4 v = *reinterpret_cast<const uint4 *>(ct + row * P + c8);
        const int gr = m0 + wm * 64 + row;
        if (gr < M) *reinterpret_cast<uint4 *>(C + (int64_t)gr * ldc + n0 + wn * 64 + c8) = v;
    }
}

// ---------------------------------------------------------------------------
// Weight gradient of the same projections: part[s][N][K] = dY[rows of split s]^T X,
// a reduction over tokens (M), split into S token ranges of whole 64-token steps so
// that the few output tiles (qkv: 9 x 7) fill the chip; the fold below sums the S
// fp32 partials in split order into the gradient and rounds once.  Both operands
// are token-major, so both MFMA operands come from the LDS image through
// ds_read_b64_tr_b16 (4 tokens x 1 column per lane, two reads per 8-token half).
// With colsum, the first column tile of each split also writes colsum[s][N] = the
// split's token sums of dY (the projection's bias gradient, from the staged image).
// The image is [64 tokens][128 columns] with 256-B rows, 16-B chunk c of row r at
// position c ^ (((r & 3) << 2) | ((r >> 2) & 3)) (conflict-free transposed reads).
// ---------------------------------------------------------------------------
typedef short bf16x4t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int tsw(int r, int c) { return r * 256 + ((c ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 4); }

// the 32 x 32 x 16 operand [32 columns from cb][16 tokens from tb] of an image: lane
// (group G = l / 16, i = 4 q + p) reads rows tb + 8 (G >> 1) + q (+ 4), columns
// cb + 16 (G & 1) + 4 p .. + 3; element j of the result is token 8 h + j of column l % 32
__device__ __forceinline__ uint4 tr_operand(uint32_t img, int tb, int cb, int lane) {
    const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int row = tb + 8 * (G >> 1) + q, col = cb + 16 * (G & 1);
    const int ch = (col >> 3) + (p >> 1), hb = 8 * (p & 1);
    const uint2 l2 = lds_rd_tr16(img + tsw(row, ch) + hb), h2 = lds_rd_tr16(img + tsw(row + 4, ch) + hb);
    return uint4{l2.x, l2.y, h2.x, h2.y};
}

template <int NS, int BK>
__global__ __launch_bounds__(kGThreads) void gemm_tn_kernel(const uint16_t *__restrict__ DY,
                                                            const uint16_t *__restrict__ X, float *__restrict__ part,
                                                            float *__restrict__ colsum, int M, int N, int K,
                                                            int64_t lddy, int64_t ldx, int S, int sps) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gl[];  // [NS buffers][dY | X]
    constexpr int SB = BK * kGT * 2, JL = BK / 16;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int ntn = N / kGT, ntk = K / kGT, tiles = ntn * ntk;
    const int s = t / tiles, tt = t - s * tiles;  // the tiles of one split share its token rows: one XCD
    const int n0 = (tt / ntk) * kGT, k0 = (tt % ntk) * kGT;
    const int steps = M / BK, st0 = s * sps, nk = max(0, min(sps, steps - st0));

    const uint16_t *dsrc[4], *xsrc[4];  // JL <= 4 used
#pragma unroll
    for (int j = 0; j < JL; ++j) {  // load u = 4 j + w: rows 4 u .. 4 u + 3, lane -> row 4 u + l / 16, position l % 16
        const int row = 4 * (4 * j + wid) + (lane >> 4), p = lane & 15;
        const int c = p ^ (((row & 3) << 2) | ((row >> 2) & 3));
        const int64_t tok = (int64_t)st0 * BK + row;
        dsrc[j] = DY + tok * lddy + n0 + c * 8;
        xsrc[j] = X + tok * ldx + k0 + c * 8;
    }
    auto stage = [=](int buf, int ks) {
        unsigned char *di = gl + buf * 2 * SB, *xi = di + SB;
#pragma unroll
        for (int j = 0; j < JL; ++j) {
            __builtin_amdgcn_global_load_lds(dsrc[j] + (int64_t)ks * BK * lddy,
                                             (__attribute__((address_space(3))) void *)(di + (4 * j + wid) * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(xsrc[j] + (int64_t)ks * BK * ldx,
                                             (__attribute__((address_space(3))) void *)(xi + (4 * j + wid) * 1024), 16, 0, 0);
        }
    };
    const int wm = wid >> 1, wn = wid & 1, h = lane >> 5;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    const uint32_t g0 = lds_off(gl);
    // colsum (the bias gradient's token sums): the first column tile of each split also sums
    // its dY image over the tokens — thread (row group rg, chunk ch) rows rg + 16 u of every
    // k-step, 8 columns, in token order; the 16 row groups meet in fixed order below
    const bool cs_on = colsum != nullptr && k0 == 0;  // workgroup-uniform
    const int cs_ch = tid & 15, cs_rg = tid >> 4;
    float cs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[e] = 0.f;
    gemm_kloop<NS, 2 * JL>(nk, stage, [&](int cur) {
        const uint32_t di = g0 + cur * 2 * SB, xi = di + SB;
        uint4 a[2][2], b[2][2];  // [k-step parity][block], as in gemm_nt_kernel
        auto rd = [&](int kk) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                a[kk & 1][i] = tr_operand(di, kk * 16, wm * 64 + i * 32, lane);
                b[kk & 1][i] = tr_operand(xi, kk * 16, wn * 64 + i * 32, lane);
            }
        };
        rd(0);
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            lgkm_wait0();
            if (kk + 1 < BK / 16) rd(kk + 1);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(a[kk & 1][i]), as_bf(b[kk & 1][j]),
                                                                        acc[i][j], 0, 0, 0);
        }
        if (cs_on) {
            uint4 v[BK / 16];
#pragma unroll
            for (int u = 0; u < BK / 16; ++u) v[u] = lds_rd128(di + tsw(cs_rg + 16 * u, cs_ch));
            lgkm_wait0();
#pragma unroll
            for (int u = 0; u < BK / 16; ++u) {
                float f[8];
                unpack16<SWH_BF16>(v[u], f);
#pragma unroll
                for (int e = 0; e < 8; ++e) cs[e] += f[e];
            }
        }
    });
    if (cs_on) {  // the stages are free (the K loop ends on a barrier): 16 row groups x 128 columns
        float *red = reinterpret_cast<float *>(gl);
#pragma unroll
        for (int e = 0; e < 8; ++e) red[cs_rg * kGT + 8 * cs_ch + e] = cs[e];
        __syncthreads();
        if (tid < kGT) {
            float v = red[tid];
#pragma unroll
            for (int r = 1; r < 16; ++r) v += red[r * kGT + tid];
            colsum[(int64_t)s * N + n0 + tid] = v;
        }
    }
    // fp32 partial: register e of block (i, j) is row n0 + 64 wm + 32 i + (e & 3) + 8 (e >> 2) + 4 h,
    // column k0 + 64 wn + 32 j + l % 32 (128 contiguous bytes per half-wave)
    float *ps = part + (int64_t)s * N * K;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int n = n0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                ps[(int64_t)n * K + k0 + wn * 64 + j * 32 + (lane & 31)] = acc[i][j][e];
            }
}

// grad[i] = round(grad[i] + sum_s part[s][i]), the sum in fp32 in split order
template <int DT>
__global__ __launch_bounds__(256) void tn_fold_kernel(const float *__restrict__ part, int S, int64_t n,
                                                      typename Elem<DT>::T *__restrict__ grad) {
    const int64_t n4 = n >> 2;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float4 a = reinterpret_cast<const float4 *>(part)[i];
        for (int s2 = 1; s2 < S; ++s2) {
            const float4 b = reinterpret_cast<const float4 *>(part + (int64_t)s2 * n)[i];
            a.x += b.x;
            a.y += b.y;
            a.z += b.z;
            a.w += b.w;
        }
        if constexpr (DT == SWH_F32) {
            float4 g = reinterpret_cast<float4 *>(grad)[i];
            g.x += a.x;
            g.y += a.y;
            g.z += a.z;
            g.w += a.w;
            reinterpret_cast<float4 *>(grad)[i] = g;
        } else {
            const uint2 g = reinterpret_cast<const uint2 *>(grad)[i];
            const float g0 = bf16_bits_to_f32(g.x & 0xffffu) + a.x, g1 = bf16_bits_to_f32(g.x >> 16) + a.y;
            const float g2 = bf16_bits_to_f32(g.y & 0xffffu) + a.z, g3 = bf16_bits_to_f32(g.y >> 16) + a.w;
            reinterpret_cast<uint2 *>(grad)[i] =
                uint2{(uint32_t)f32_to_bf16_bits(g0) | ((uint32_t)f32_to_bf16_bits(g1) << 16),
                      (uint32_t)f32_to_bf16_bits(g2) | ((uint32_t)f32_to_bf16_bits(g3) << 16)};
        }
    }
}

}  // namespace
}  // namespace swh

using namespace swh;

template <int NS, int BK>
static int launch_nt(const void *A, const void *B, const void *bias, void *C, int64_t M, int64_t N, int64_t K,
                     int64_t lda, int64_t ldb, int64_t ldc, int64_t tiles, hipStream_t s) {
    constexpr int lds = NS * 2 * kGT * BK * 2;
    if (!lds_opt_in<&gemm_nt_kernel<true, NS, BK>>() || !lds_opt_in<&gemm_nt_kernel<false, NS, BK>>())
        return SWH_E_LAUNCH;
    if (bias)
        gemm_nt_kernel<true, NS, BK><<<(unsigned)tiles, kGThreads, lds, s>>>(
            static_cast<const uint16_t *>(A), static_cast<const uint16_t *>(B), static_cast<const uint16_t *>(bias),
            static_cast<uint16_t *>(C), (int)M, (int)N, (int)K, lda, ldb, ldc);
    else
        gemm_nt_kernel<false, NS, BK><<<(unsigned)tiles, kGThreads, lds, s>>>(
            static_cast<const uint16_t *>(A), static_cast<const uint16_t *>(B), nullptr, static_cast<uint16_t *>(C),
            (int)M, (int)N, (int)K, lda, ldb, ldc);
    return launch_status();
}

extern "C" int swh_gemm_nt(const void *A, const void *B, const void *bias, void *C, int64_t M, int64_t N, int64_t K,
                           int64_t lda, int64_t ldb, int64_t ldc, void *stream) {
    if (!A || !B || !C || M < 0 || N < 0 || K <= 0) return SWH_E_ARG;
    if (N % kGT || K % kGK || lda < K || ldb < K || ldc < N || lda % 8 || ldb % 8 || ldc % 8) return SWH_E_ARG;
    if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B) | reinterpret_cast<uintptr_t>(C)) & 15)
        return SWH_E_ARG;
    if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return SWH_E_ARG;
    if (M == 0 || N == 0) return SWH_OK;
    const int64_t tiles = ((M + kGT - 1) / kGT) * (N / kGT);
    if (tiles > INT32_MAX) return SWH_E_ARG;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return launch_nt<2, 64>(A, B, bias, C, M, N, K, lda, ldb, ldc, tiles, s);
}

template <int NS, int BK>
static int launch_tn(const void *dY, const void *X, float *part, float *colsum, int64_t M, int64_t N, int64_t K,
                     int64_t lddy, int64_t ldx, int S, int64_t grid, hipStream_t s) {
    constexpr int lds = NS * 2 * kGT * BK * 2;
    if (!lds_opt_in<&gemm_tn_kernel<NS, BK>>()) return SWH_E_LAUNCH;
    const int steps = (int)(M / BK), sps = (steps + S - 1) / S;
    gemm_tn_kernel<NS, BK><<<(unsigned)grid, kGThreads, lds, s>>>(static_cast<const uint16_t *>(dY),
                                                                   static_cast<const uint16_t *>(X), part, colsum,
                                                                   (int)M, (int)N, (int)K, lddy, ldx, S,
                                                                   sps > 1 ? sps : 1);
    return launch_status();
}

extern "C" int swh_gemm_tn_partials(const void *dY, const void *X, float *part, float *colsum, int64_t M, int64_t N,
                                    int64_t K, int64_t lddy, int64_t ldx, int32_t S, void *stream) {
    if (!dY || !X || !part || M < 0 || S < 1 || N <= 0 || K <= 0) return SWH_E_ARG;
    if (M % kGK || N % kGT || K % kGT || lddy < N || ldx < K || lddy % 8 || ldx % 8) return SWH_E_ARG;
    if ((reinterpret_cast<uintptr_t>(dY) | reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(part)) & 15)
        return SWH_E_ARG;
    if (colsum && (reinterpret_cast<uintptr_t>(colsum) & 3)) return SWH_E_ARG;
    if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX || S > 1024) return SWH_E_ARG;
    const int64_t grid = (N / kGT) * (K / kGT) * (int64_t)S;
    if (grid > INT32_MAX) return SWH_E_ARG;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return launch_tn<2, 64>(dY, X, part, colsum, M, N, K, lddy, ldx, S, grid, s);
}

extern "C" int swh_gemm_tn_fold(const float *part, int32_t S, int64_t n, void *grad, int32_t dtype, void *stream) {
    if (!part || !grad || S < 1 || n < 0 || n % 4) return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F32) return SWH_E_DTYPE;
    if ((reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(grad)) & (dtype == SWH_F32 ? 15 : 7))
        return SWH_E_ARG;
    if (n == 0) return SWH_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t n4 = n / 4;
    const int64_t nb0 = (n4 + 255) / 256;
    const unsigned nb = (unsigned)(nb0 < 2048 ? nb0 : 2048);
    if (dtype == SWH_BF16)
        tn_fold_kernel<SWH_BF16><<<nb, 256, 0, s>>>(part, S, n, static_cast<uint16_t *>(grad));
    else
        tn_fold_kernel<SWH_F32><<<nb, 256, 0, s>>>(part, S, n, static_cast<float *>(grad));
    return launch_status();
}
