// C[M, N] = A[M, K] · B[N, K]^T (+ bias[N]) for the wide training projections
// (gate/up forward, the lm head, the down input gradient through a transposed
// weight copy), where csrc/tgemm.hip's 128 x 128 two-stage loop reaches 0.7
// PFLOP/s and hipBLASLt 1.0-1.1.
//
// 256 x 256 output tiles, 8 waves of 128 x 64 (2 along M x 4 along N) on
// v_mfma_f32_16x16x32_bf16, 64-wide K tiles staged by LDS-DMA (global_load_lds,
// 16 B per lane) into two 64 KB buffers (one workgroup per CU).  Each K tile is
// four phases, one per quadrant (64 rows x 32 columns) of a wave's output:
//
//   phase   LDS reads (this tile)      MFMAs          restage (region freed a phase ago)
//   0       A rows 0-63, B cols 0-31   (top, left)    B cols 0-31 of tile t+1 (other buffer)
//   1       B cols 32-63               (top, right)   A rows 0-63 of tile t+2 (this buffer)
//   2       A rows 64-127              (bottom,right) B cols 32-63 of tile t+2
//   3       B cols 0-31 (again)        (bottom, left) A rows 64-127 of tile t+2
//
// (rows / columns relative to the wave's 128 x 64 block).  Every phase opens on a
// raw s_barrier, so a region is restaged only after every wave's reads of it
// retired (each wave waits lgkmcnt(0) before its MFMAs); phase 0 first waits with
// a counted vmcnt for the last region of its tile (the 6 loads issued after it
// stay in flight, never vmcnt(0) in the steady state), so every load has 4-7
// phases of MFMA work to land under.  Both operands are read with the same
// 16 x 32 fragment load (row = lane % 16, 8 k per lane); the weight fragment is
// the MFMA's first operand, so a lane's 4 accumulators are 4 consecutive output
// columns of one row (8-B stores).  The K order of every sum is fixed (16-k MFMA
// steps in ascending k), and a row's result does not depend on the tile it falls in.
#include "common.hpp"

namespace swh {
namespace {

constexpr int kT = 256;          // tile rows = tile columns
constexpr int kBK = 64;          // K tile
constexpr int kThreads = 512;
constexpr int kImg = kT * kBK * 2;  // one operand's K-tile image: 32 KB, [256 rows][128 B]
constexpr int kBuf = 2 * kImg;      // A image | B image
constexpr int kLds = 2 * kBuf;      // two buffers: 128 KB
constexpr int kGroupM = 8;          // row blocks per tile group (L2 reuse of the B blocks)

typedef float f32x4t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8t __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lds_u32(const unsigned char *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char *)p;
}
template <int OFF>
__device__ __forceinline__ u32x4t ds128(uint32_t base) {
    u32x4t v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(OFF));
    return v;
}
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void phase_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void lgkm_wait() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ bf16x8t bf(const u32x4t &v) { return __builtin_bit_cast(bf16x8t, v); }

// A fragments of one half (IH) of the wave's 128 rows: 4 row groups x 2 k-steps
template <int IH>
__device__ __forceinline__ void read_a(uint32_t b0, uint32_t b1, u32x4t (&a)[4][2]) {
    constexpr int R = IH * 64 * 128;
    a[0][0] = ds128<R + 0 * 2048>(b0);
    a[0][1] = ds128<R + 0 * 2048>(b1);
    a[1][0] = ds128<R + 1 * 2048>(b0);
    a[1][1] = ds128<R + 1 * 2048>(b1);
    a[2][0] = ds128<R + 2 * 2048>(b0);
    a[2][1] = ds128<R + 2 * 2048>(b1);
    a[3][0] = ds128<R + 3 * 2048>(b0);
    a[3][1] = ds128<R + 3 * 2048>(b1);
}
// B fragments of one half (JH) of the wave's 64 columns: 2 column groups x 2 k-steps
template <int JH>
__device__ __forceinline__ void read_b(uint32_t b0, uint32_t b1, u32x4t (&b)[2][2]) {
    constexpr int R = JH * 32 * 128;
    b[0][0] = ds128<R + 0 * 2048>(b0);
    b[0][1] = ds128<R + 0 * 2048>(b1);
    b[1][0] = ds128<R + 1 * 2048>(b0);
    b[1][1] = ds128<R + 1 * 2048>(b1);
}
template <int IH, int JH>
__device__ __forceinline__ void mma_quadrant(f32x4t (&acc)[8][4], const u32x4t (&a)[4][2], const u32x4t (&b)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                acc[IH * 4 + i][JH * 2 + j] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf(b[j][kk]), bf(a[i][kk]), acc[IH * 4 + i][JH * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
}

template <bool BIAS>
__global__ __launch_bounds__(kThreads) void gemm_nt256_kernel(const uint16_t *__restrict__ A,
                                                              const uint16_t *__restrict__ B,
                                                              const uint16_t *__restrict__ bias,
                                                              uint16_t *__restrict__ C, int M, int N, int K, int lda,
                                                              int ldb, int64_t ldc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gl[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // XCD-contiguous tile ranges (bijective remap), then groups of kGroupM row blocks
    // x all column blocks, row block fastest: the ~32 workgroups an XCD runs at once
    // share 8 A row blocks and 4 B column blocks in its L2
    const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int tm = (M + kT - 1) / kT, tn = (N + kT - 1) / kT;
    const int grp = t / (kGroupM * tn), first = grp * kGroupM, gsz = min(tm - first, kGroupM);
    const int tg = t - grp * kGroupM * tn;
    const int m0 = (first + tg % gsz) * kT, n0 = (tg / gsz) * kT;
    const int nk = K / kBK;

    // staging: part p of a K tile is two rounds of 8 waves x 1 KB (8 image rows per wave);
    // lane l fills image row 8 rb + l / 8 at 16-B position l % 8 with source chunk
    // (l % 8) ^ ((row >> 1) & 7) (the bank swizzle, undone on the fragment reads)
    //   part 0: B rows {0-31, 64-95, 128-159, 192-223}   part 1: A rows {0-63, 128-191}
    //   part 2: B rows {32-63, 96-127, 160-191, 224-255} part 3: A rows {64-127, 192-255}
    int rbk[4][2];
    {
        const int bq = (w >> 2) * 8 + (w & 3);
        rbk[0][0] = bq;
        rbk[0][1] = 16 + bq;
        rbk[1][0] = w;
        rbk[1][1] = 16 + w;
        rbk[2][0] = 4 + bq;
        rbk[2][1] = 20 + bq;
        rbk[3][0] = 8 + w;
        rbk[3][1] = 24 + w;
    }
    uint32_t so[4][2];  // element offsets of this lane's source chunk (k = 0)
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = rbk[p][h] * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
            so[p][h] = (p & 1) ? (uint32_t)min(m0 + row, M - 1) * (uint32_t)lda + c * 8
                               : (uint32_t)min(n0 + row, N - 1) * (uint32_t)ldb + c * 8;
        }
    auto stage = [&](int p, int buf, int kt) {
        const uint16_t *src = (p & 1) ? A : B;
        unsigned char *img = gl + buf * kBuf + ((p & 1) ? 0 : kImg);
        const int k0 = kt * kBK;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            __builtin_amdgcn_global_load_lds(src + so[p][h] + k0,
                                             (__attribute__((address_space(3))) void *)(img + rbk[p][h] * 1024), 16, 0, 0);
    };

    // fragment read bases: row 16 g + lane % 16 of a 16-row group, chunk 4 kk + lane / 16
    const int wr = w >> 2, wc = w & 3, fr = lane & 15, sw = fr >> 1;
    const uint32_t g0 = lds_u32(gl);
    uint32_t ba[2][2], bb[2][2];  // [buffer][kk]
#pragma unroll
    for (int bu = 0; bu < 2; ++bu)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const uint32_t o = fr * 128 + ((((kk * 4) + (lane >> 4)) ^ sw) << 4);
            ba[bu][kk] = g0 + bu * kBuf + wr * 128 * 128 + o;
            bb[bu][kk] = g0 + bu * kBuf + kImg + wc * 64 * 128 + o;
        }

    f32x4t acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4t{0.f, 0.f, 0.f, 0.f};
    u32x4t fa[2][4][2], fb[2][2];

    // prologue: tiles 0 and 1, every part
#pragma unroll
    for (int p = 0; p < 4; ++p) stage(p, 0, 0);
    if (nk > 1) {
#pragma unroll
        for (int p = 0; p < 4; ++p) stage(p, 1, 1);
    }
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const uint32_t a0 = cur ? ba[1][0] : ba[0][0], a1 = cur ? ba[1][1] : ba[0][1];
        const uint32_t b0 = cur ? bb[1][0] : bb[0][0], b1 = cur ? bb[1][1] : bb[0][1];
        const bool more1 = kt + 1 < nk, more2 = kt + 2 < nk;
        // phase 0: this tile's parts have landed (the 6 loads of tile kt + 1 issued after
        // its last part stay in flight; at kt = 0 the 8 prologue loads of tile 1)
        if (more1) {
            if (kt == 0) vm_wait<8>();
            else vm_wait<6>();
        } else {
            vm_wait<0>();
        }
        phase_barrier();
        read_a<0>(a0, a1, fa[0]);
        read_b<0>(b0, b1, fb);
        if (kt >= 1 && more1) stage(0, cur ^ 1, kt + 1);
        lgkm_wait();
        mma_quadrant<0, 0>(acc, fa[0], fb);
        // phase 1
        phase_barrier();
        read_b<1>(b0, b1, fb);
        if (more2) stage(1, cur, kt + 2);
        lgkm_wait();
        mma_quadrant<0, 1>(acc, fa[0], fb);
        // phase 2
        phase_barrier();
        read_a<1>(a0, a1, fa[1]);
        if (more2) stage(2, cur, kt + 2);
        lgkm_wait();
        mma_quadrant<1, 1>(acc, fa[1], fb);
        // phase 3
        phase_barrier();
        read_b<0>(b0, b1, fb);
        if (more2) stage(3, cur, kt + 2);
        lgkm_wait();
        mma_quadrant<1, 0>(acc, fa[1], fb);
    }

    // epilogue: accumulator (i, j) of lane l holds C[row 16 i + l % 16][cols 16 j + 4 (l / 16) .. + 3]
    // of the wave's 128 x 64 block
    const int mrow = m0 + wr * 128 + fr, ncol = n0 + wc * 64 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = ncol + 16 * j;
        if (n >= N) continue;
        float bz[4] = {0.f, 0.f, 0.f, 0.f};
        if (BIAS) {
            const uint2 bv = *reinterpret_cast<const uint2 *>(bias + n);
            bz[0] = bf16_bits_to_f32(bv.x & 0xffffu);
            bz[1] = bf16_bits_to_f32(bv.x >> 16);
            bz[2] = bf16_bits_to_f32(bv.y & 0xffffu);
            bz[3] = bf16_bits_to_f32(bv.y >> 16);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int m = mrow + 16 * i;
            if (m >= M) continue;
            const f32x4t v = acc[i][j];
            const uint2 o{(uint32_t)f32_to_bf16_bits(v[0] + bz[0]) | ((uint32_t)f32_to_bf16_bits(v[1] + bz[1]) << 16),
                          (uint32_t)f32_to_bf16_bits(v[2] + bz[2]) | ((uint32_t)f32_to_bf16_bits(v[3] + bz[3]) << 16)};
            *reinterpret_cast<uint2 *>(C + (int64_t)m * ldc + n) = o;
        }
    }
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int swh_gemm_nt256(const void *A, const void *B, const void *bias, void *C, int64_t M, int64_t N, int64_t K,
                              int64_t lda, int64_t ldb, int64_t ldc, void *stream) {
    if (!A || !B || !C || M < 0 || N < 0 || K <= 0) return SWH_E_ARG;
    if (N % 8 || K % kBK || lda < K || ldb < K || ldc < N || lda % 8 || ldb % 8 || ldc % 4) return SWH_E_ARG;
    if (((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) || (reinterpret_cast<uintptr_t>(C) & 7))
        return SWH_E_ARG;
    if (bias && (reinterpret_cast<uintptr_t>(bias) & 7)) return SWH_E_ARG;
    // 32-bit element offsets of the staged rows
    if (M * lda > (int64_t)UINT32_MAX || N * ldb > (int64_t)UINT32_MAX || lda > INT32_MAX || ldb > INT32_MAX)
        return SWH_E_ARG;
    if (M == 0 || N == 0) return SWH_OK;
    const int64_t tiles = ((M + kT - 1) / kT) * ((N + kT - 1) / kT);
    if (tiles > INT32_MAX) return SWH_E_ARG;
    if (!lds_opt_in<&gemm_nt256_kernel<true>>() || !lds_opt_in<&gemm_nt256_kernel<false>>()) return SWH_E_LAUNCH;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (bias)
        gemm_nt256_kernel<true><<<(unsigned)tiles, kThreads, kLds, s>>>(
            static_cast<const uint16_t *>(A), static_cast<const uint16_t *>(B), static_cast<const uint16_t *>(bias),
            static_cast<uint16_t *>(C), (int)M, (int)N, (int)K, (int)lda, (int)ldb, ldc);
    else
        gemm_nt256_kernel<false><<<(unsigned)tiles, kThreads, kLds, s>>>(
            static_cast<const uint16_t *>(A), static_cast<const uint16_t *>(B), nullptr, static_cast<uint16_t *>(C),
            (int)M, (int)N, (int)K, (int)lda, (int)ldb, ldc);
    return launch_status();
}
