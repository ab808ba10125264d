// C[M, N] = A[M, K] · B[N, K]^T (+ bias[N]) and the token-split weight gradient
// dY^T X for the wide training projections (gate/up forward, the lm head, the down
// input gradient through a transposed weight copy), where csrc/tgemm.hip's
// 128 x 128 two-stage loop reaches 0.7 PFLOP/s and hipBLASLt 1.0-1.1.  Measured
// (DESIGN.md §14e): 1.32 PFLOP/s at 8192^3, but slower than hipBLASLt at the bench
// step's K = 896 shapes and at par on the weight gradients, so the engine does not
// route to these entry points; they stay as tested kernels with tools/bench_nt256.py.
//
// 256 x 256 output tiles, 8 waves of 128 x 64 (2 along M x 4 along N) on
// v_mfma_f32_16x16x32_bf16, 64-wide K tiles staged by LDS-DMA (buffer_load ... lds
// through one buffer descriptor per staged run, 16 B per lane) into two 64 KB
// buffers (one workgroup per CU).  A K tile is four
// phases, one per quadrant (64 rows x 32 columns) of a wave's 128 x 64 block, in
// the order (top, left), (top, right), (bottom, right), (bottom, left), so each
// phase changes one operand half.  Every phase: raw s_barrier, the LDS fragment
// reads of a LATER quadrant (into the other register half), one restaged part,
// the 16 MFMAs of this quadrant on fragments read a phase earlier, lgkmcnt(0):
//
//   phase  reads (into registers)          restages (into this tile's buffer)
//   0      B cols 32-63 of tile t          A rows 0-63   of tile t+2
//   1      A rows 64-127 of tile t         B cols 32-63  of tile t+2
//   2      A rows 0-63 of tile t+1         A rows 64-127 of tile t+2
//   3      B cols 0-31 of tile t+1         B cols 0-31   of tile t+2
//
// (rows / columns relative to the wave's block; each part is the union over the
// waves).  A region is restaged a phase after its last read (the barrier follows
// every wave's lgkmcnt(0)), and phases 2 and 3 first wait with a counted vmcnt
// for the part they read (10 / 6 later loads stay in flight; never vmcnt(0) in
// the steady state), so a load has 4-7 phases to land.  The B-fragment register
// halves alternate from tile to tile (the loop runs tiles in pairs).  Both
// operands use the same 16 x 32 fragment read (row = lane % 16, 8 k per lane); the
// weight fragment is the MFMA's first operand, so a lane's 4 accumulators are 4
// consecutive output columns of one row (8-B stores).  Every sum runs in
// ascending K (16-k MFMA steps), so a row's result does not depend on its tile.
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
typedef uint32_t u32x2t __attribute__((ext_vector_type(2)));

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

template <int V>
using ic = std::integral_constant<int, V>;

// The eight-phase K loop shared by the NT and TN kernels (schedule: file header).
// stage(p, buf, kt) restages part p of K tile kt into buffer buf; read_a(ic<IH>, buf,
// fa[h]) / read_b(ic<JH>, buf, fb[h]) read one operand half's fragments of the tile
// in buffer buf.  Parts: 0 = A top, 1 = B right, 2 = A bottom, 3 = B left.
template <class Stage, class ReadA, class ReadB>
__device__ __forceinline__ void eight_phase_loop(int nk, f32x4t (&acc)[8][4], Stage stage, ReadA read_a, ReadB read_b) {
    u32x4t fa[2][4][2], fb[2][2][2];  // A [top / bottom], B [alternating half][column group][kk]
    // prologue: tiles 0 and 1, parts in issue order 0..3; the first quadrant's fragments
#pragma unroll
    for (int p = 0; p < 4; ++p) stage(p, 0, 0);
    if (nk > 1) {
#pragma unroll
        for (int p = 0; p < 4; ++p) stage(p, 1, 1);
        vm_wait<8>();
    } else {
        vm_wait<0>();
    }
    phase_barrier();
    read_a(ic<0>{}, 0, fa[0]);
    read_b(ic<0>{}, 0, fb[0]);
    lgkm_wait();

    // one K tile; BS = the register half holding its left B fragments
    auto tile = [&](int kt, auto bs_tag) {
        constexpr int BS = decltype(bs_tag)::value;
        const int cur = kt & 1, nxt = cur ^ 1;
        const bool more1 = kt + 1 < nk, more2 = kt + 2 < nk;
        // phase 0: (top, left); read (top, right)
        phase_barrier();
        read_b(ic<1>{}, cur, fb[BS ^ 1]);
        if (more2) stage(0, cur, kt + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma_quadrant<0, 0>(acc, fa[0], fb[BS]);
        lgkm_wait();
        // phase 1: (top, right); read the bottom A half
        phase_barrier();
        read_a(ic<1>{}, cur, fa[1]);
        if (more2) stage(1, cur, kt + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma_quadrant<0, 1>(acc, fa[0], fb[BS ^ 1]);
        lgkm_wait();
        // phase 2: (bottom, right); read the next tile's top A half
        if (more1) {
            if (more2) vm_wait<10>();
            else vm_wait<6>();
        }
        phase_barrier();
        if (more1) read_a(ic<0>{}, nxt, fa[0]);
        if (more2) stage(2, cur, kt + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma_quadrant<1, 1>(acc, fa[1], fb[BS ^ 1]);
        lgkm_wait();
        // phase 3: (bottom, left); read the next tile's left B half
        if (more1) {
            if (more2) vm_wait<6>();
            else vm_wait<0>();
        }
        phase_barrier();
        if (more1) read_b(ic<0>{}, nxt, fb[BS ^ 1]);
        if (more2) stage(3, cur, kt + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma_quadrant<1, 0>(acc, fa[1], fb[BS]);
        lgkm_wait();
    };
    for (int kt = 0; kt < nk; kt += 2) {
        tile(kt, ic<0>{});
        if (kt + 1 < nk) tile(kt + 1, ic<1>{});
    }
}

template <bool BIAS>
__global__ __launch_bounds__(kThreads) void gemm_nt256_kernel(const uint16_t *__restrict__ A,
                                                              const uint16_t *__restrict__ B,
                                                              const uint16_t *__restrict__ bias,
                                                              uint16_t *__restrict__ C, int M, int N, int K, int lda,
                                                              int ldb, int64_t ldc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gl[];
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
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
    //   part 0: A rows {0-63, 128-191}   part 1: B rows {32-63, 96-127, 160-191, 224-255}
    //   part 2: A rows {64-127, 192-255} part 3: B rows {0-31, 64-95, 128-159, 192-223}
    int rbk[4][2];
    {
        const int bq = (w >> 2) * 8 + (w & 3);
        rbk[0][0] = w;
        rbk[0][1] = 16 + w;
        rbk[1][0] = 4 + bq;
        rbk[1][1] = 20 + bq;
        rbk[2][0] = 8 + w;
        rbk[2][1] = 24 + w;
        rbk[3][0] = bq;
        rbk[3][1] = 16 + bq;
    }
    // one buffer descriptor per (part, round): base = the round's first row, records =
    // the bytes up to the operand's last row, so rows past M / N are dropped by the range
    // check (their LDS rows feed only outputs that are never stored); the lane's row in
    // the 8-row block and its chunk go in the VGPR offset, the K offset in the SGPR one.
    // The chunk swizzle depends on the row block's parity only, which is the wave's.
    __amdgpu_buffer_rsrc_t rs[4][2];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool isb = p & 1;
            const int row0 = (isb ? n0 : m0) + rbk[p][h] * 8, left = (isb ? N : M) - row0;
            const int ld = isb ? ldb : lda;
            const uint16_t *base = left > 0 ? (isb ? B : A) + (int64_t)row0 * ld : (isb ? B : A);
            rs[p][h] = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, left > 0 ? left * ld * 2 : 0, 0x00020000);
        }
    const int chunk = (lane & 7) ^ (((w & 1) * 4 + (lane >> 4)) & 7);
    const int voa = (lane >> 3) * lda * 2 + chunk * 16, vob = (lane >> 3) * ldb * 2 + chunk * 16;
    auto stage = [&](int p, int buf, int kt) {
        unsigned char *img = gl + buf * kBuf + ((p & 1) ? kImg : 0);
#pragma unroll
        for (int h = 0; h < 2; ++h)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs[p][h],
                                                     (__attribute__((address_space(3))) void *)(img + rbk[p][h] * 1024), 16,
                                                     (p & 1) ? vob : voa, kt * kBK * 2, 0, 0);
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
    eight_phase_loop(
        nk, acc, stage,
        [&](auto ih, int buf, u32x4t (&f)[4][2]) { read_a<decltype(ih)::value>(ba[buf][0], ba[buf][1], f); },
        [&](auto jh, int buf, u32x4t (&f)[2][2]) { read_b<decltype(jh)::value>(bb[buf][0], bb[buf][1], f); });

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

// ---------------------------------------------------------------------------
// Weight gradient of the same projections: part[s][N][K] = dY[tokens of split s]^T X
// (fp32, folded by swh_gemm_tn_fold), on the same schedule.  The contraction runs
// over tokens, which are the ROWS of both operands, so the K tile is 64 tokens and
// the images are [64 tokens][256 columns], read through ds_read_b64_tr_b16 (per
// 16-lane group a 4-token x 16-column block, delivered column-major: two reads give
// a lane the 8 tokens of one column that a 16 x 32 MFMA fragment needs).  Image of
// one operand: two 16 KB halves (columns 0-127, 128-255), each eight 2 KB groups of
// 8 tokens, each group four 512-B column slots of 32 columns: token r of the group at
// 64 (r % 8), its 16-B chunk c (of the slot) at 16 (c ^ ((r / 4) % 4)).  dY (the "A"
// operand, the N side) keeps column slots in order; X (the "B" side) stores its
// 32-column slots in the order 0, 2, 1, 3, so that a wave's left / right 32 columns
// of either 64-column half are the first / second 1 KB of every group: each part of
// the schedule is again 16 contiguous 1 KB runs.
// ---------------------------------------------------------------------------
template <int OFF>
__device__ __forceinline__ uint2 tr_read(uint32_t base) {
    u32x2t v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(OFF));
    return uint2{v.x, v.y};
}
// fragment (16 columns, 32 tokens): lo = tokens 8 (l / 16) .. + 3, hi = + 4 .. + 7
template <int OFF>
__device__ __forceinline__ u32x4t tr_frag(uint32_t blo, uint32_t bhi) {
    const uint2 lo = tr_read<OFF>(blo), hi = tr_read<OFF>(bhi);
    return u32x4t{lo.x, lo.y, hi.x, hi.y};
}

__global__ __launch_bounds__(kThreads) void gemm_tn256_kernel(const uint16_t *__restrict__ DY,
                                                              const uint16_t *__restrict__ X, float *__restrict__ part,
                                                              int M, int N, int K, int lddy, int ldx, int S, int sps) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gl[];
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    // XCD-contiguous ranges; the tiles of one split (same tokens) are consecutive
    const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int tn = (N + kT - 1) / kT, tk = (K + kT - 1) / kT, tiles = tn * tk;
    const int s = t / tiles, tt = t - s * tiles;
    const int n0 = (tt / tk) * kT, k0 = (tt % tk) * kT;
    const int steps = M / kBK, st0 = s * sps, nk = max(0, min(sps, steps - st0));
    const int tok0 = st0 * kBK;

    // staging: part p, round h (image half h) -> wave w fills group w (tokens 8 w .. 8 w + 7),
    // 1 KB run hf (slots 2 hf, 2 hf + 1); lane l -> slot 2 hf + l / 32, token r = (l / 4) % 8,
    // position l % 4 holding chunk (l % 4) ^ (((8 w + r) / 4) % 4)
    __amdgpu_buffer_rsrc_t rs[4][2];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool isb = p & 1;
            const int ld = isb ? ldx : lddy, cols = isb ? K : N, c0 = (isb ? k0 : n0) + h * 128;
            const int64_t first = (int64_t)(tok0 + 8 * w) * ld + c0, last = (int64_t)(M - 1) * ld + cols;
            const uint16_t *src = isb ? X : DY;
            rs[p][h] = __builtin_amdgcn_make_buffer_rsrc((void *)(src + (first < last ? first : 0)), (short)0,
                                                         first < last ? (int)((last - first) * 2) : 0, 0x00020000);
        }
    int vo[2][2];  // [operand][run hf]: lane's byte offset within its 8-token group
    {
        const int r = (lane >> 2) & 7, slot_lo = lane >> 5;
        const int ch = (lane & 3) ^ (((8 * w + r) >> 2) & 3);
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int slot = 2 * hf + slot_lo;
            const int sta = slot, stb = (slot == 1) ? 2 : (slot == 2) ? 1 : slot;  // X: slots hold 32-col blocks 0,2,1,3
            vo[0][hf] = r * lddy * 2 + (sta * 32 + ch * 8) * 2;
            vo[1][hf] = r * ldx * 2 + (stb * 32 + ch * 8) * 2;
        }
    }
    auto stage = [&](int p, int buf, int kt) {
        const bool isb = p & 1;
        const int hf = (p == 1 || p == 2) ? 1 : 0;
        const int ld = isb ? ldx : lddy;
        // operand images: dY of buffer b at 32 KB b, X at 64 KB + 32 KB b
        unsigned char *img = gl + (isb ? 2 * kImg : 0) + buf * kImg;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs[p][h],
                                                     (__attribute__((address_space(3))) void *)(img + h * 16384 + w * 2048 + hf * 1024),
                                                     16, vo[isb][hf], kt * kBK * ld * 2, 0, 0);
    };

    // transposed fragment reads: lane (g = l / 16, q = (l / 4) % 4, p = l % 4) reads token
    // 8 g + q (+ 4) of kk, columns 4 p .. 4 p + 3 of a 16-column block; the lane-dependent
    // part of the address: 2048 g + 64 (4 hi + q) + 16 ((blk1 ^ (g & 1)) * 2 + ((p >> 1) ^ hi)) + 8 (p & 1)
    // with blk1 = the block's 16-column parity within its slot (bit 1 of its chunk)
    const int wr = w >> 2, wc = w & 3, g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const uint32_t g0 = lds_u32(gl);
    uint32_t bt[2][2][2];  // [operand][hi][blk1]
#pragma unroll
    for (int hi = 0; hi < 2; ++hi)
#pragma unroll
        for (int b1 = 0; b1 < 2; ++b1) {
            const uint32_t o = 2048 * g + 64 * (4 * hi + q) + 16 * (((b1 ^ (g & 1)) << 1) | ((pp >> 1) ^ hi)) + 8 * (pp & 1);
            bt[0][hi][b1] = g0 + wr * 16384 + o;                                // dY: columns 128 wr ..
            bt[1][hi][b1] = g0 + 2 * kImg + (wc >> 1) * 16384 + (wc & 1) * 512 + o;  // X: 64-col half wc
        }
    // dY half IH of the wave's 128 columns: block i (16 columns) in slot 2 IH + i / 2, parity i % 2
    auto read_dy = [&](auto ih, int buf, u32x4t (&f)[4][2]) {
        constexpr int IH = decltype(ih)::value;
        const uint32_t b00 = bt[0][0][0] + buf * kImg, b10 = bt[0][1][0] + buf * kImg;
        const uint32_t b01 = bt[0][0][1] + buf * kImg, b11 = bt[0][1][1] + buf * kImg;
        f[0][0] = tr_frag<(2 * IH + 0) * 512>(b00, b10);
        f[1][0] = tr_frag<(2 * IH + 0) * 512>(b01, b11);
        f[2][0] = tr_frag<(2 * IH + 1) * 512>(b00, b10);
        f[3][0] = tr_frag<(2 * IH + 1) * 512>(b01, b11);
        f[0][1] = tr_frag<(2 * IH + 0) * 512 + 8192>(b00, b10);
        f[1][1] = tr_frag<(2 * IH + 0) * 512 + 8192>(b01, b11);
        f[2][1] = tr_frag<(2 * IH + 1) * 512 + 8192>(b00, b10);
        f[3][1] = tr_frag<(2 * IH + 1) * 512 + 8192>(b01, b11);
    };
    // X half JH of the wave's 64 columns: slot 2 JH + (wc & 1) (in the base), blocks j = parity
    auto read_x = [&](auto jh, int buf, u32x4t (&f)[2][2]) {
        constexpr int JH = decltype(jh)::value;
        const uint32_t b00 = bt[1][0][0] + buf * kImg, b10 = bt[1][1][0] + buf * kImg;
        const uint32_t b01 = bt[1][0][1] + buf * kImg, b11 = bt[1][1][1] + buf * kImg;
        f[0][0] = tr_frag<JH * 1024>(b00, b10);
        f[1][0] = tr_frag<JH * 1024>(b01, b11);
        f[0][1] = tr_frag<JH * 1024 + 8192>(b00, b10);
        f[1][1] = tr_frag<JH * 1024 + 8192>(b01, b11);
    };

    f32x4t acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4t{0.f, 0.f, 0.f, 0.f};
    if (nk > 0) eight_phase_loop(nk, acc, stage, read_dy, read_x);

    // accumulator (i, j) of lane l: dW[row 16 i + l % 16 of the wave's 128 N rows]
    // [columns 16 j + 4 (l / 16) .. + 3 of its 64 K columns], fp32, 16-B stores
    float *ps = part + (int64_t)s * N * K;
    const int nrow = n0 + wr * 128 + (lane & 15), kcol = k0 + wc * 64 + 4 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = kcol + 16 * j;
        if (k >= K) continue;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int n = nrow + 16 * i;
            if (n < N) *reinterpret_cast<f32x4t *>(ps + (int64_t)n * K + k) = acc[i][j];
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
    // 32-bit byte offsets and record counts of the buffer descriptors
    if (M * lda * 2 > (int64_t)INT32_MAX || N * ldb * 2 > (int64_t)INT32_MAX) return SWH_E_ARG;
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

extern "C" int swh_gemm_tn256_partials(const void *dY, const void *X, float *part, int64_t M, int64_t N, int64_t K,
                                       int64_t lddy, int64_t ldx, int32_t S, void *stream) {
    if (!dY || !X || !part || M < 0 || S < 1 || N <= 0 || K <= 0) return SWH_E_ARG;
    if (M % kBK || N % 16 || K % 16 || lddy < N || ldx < K || lddy % 8 || ldx % 8) return SWH_E_ARG;
    if ((reinterpret_cast<uintptr_t>(dY) | reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(part)) & 15)
        return SWH_E_ARG;
    if (M * lddy * 2 > (int64_t)INT32_MAX || M * ldx * 2 > (int64_t)INT32_MAX || S > 1024) return SWH_E_ARG;
    const int64_t grid = ((N + kT - 1) / kT) * ((K + kT - 1) / kT) * (int64_t)S;
    if (grid > INT32_MAX) return SWH_E_ARG;
    if (!lds_opt_in<&gemm_tn256_kernel>()) return SWH_E_LAUNCH;
    const int steps = (int)(M / kBK), sps = steps > 0 ? (steps + S - 1) / S : 1;
    gemm_tn256_kernel<<<(unsigned)grid, kThreads, kLds, reinterpret_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(dY), static_cast<const uint16_t *>(X), part, (int)M, (int)N, (int)K, (int)lddy,
        (int)ldx, S, sps);
    return launch_status();
}
