// Decode-step kernels of the rollout engine (batch <= 64 rows per tile):
//
//  * swh_decode_gemm — weight-streaming "skinny" GEMM  Y[M,N] = X[M,K] W[N,K]^T
//    on MFMA v_mfma_f32_16x16x32_bf16, with the decoder's neighbours fused:
//      prologue  RMSNorm of X (Qwen2RMSNorm rounding points)      [qkv, gate_up, lm head]
//      epilogue  + bias                                           [qkv]
//                residual: s = bf16(s + bf16(acc)) in place       [o_proj, down_proj]
//                          + per-row sums of squares of the new s (the next RMSNorm)
//                SiLU gate: y = bf16(bf16(silu(bf16 g)) * bf16 u) [gate_up]
//    A workgroup owns all 64 rows x NB = 16*CB output columns of one K slice;
//    its NW waves (4/8/16) split the slice's k-steps and each wave issues ALL
//    the weight/X loads of a round of U k-steps at once (one HBM round trip
//    per round, tail clamped rather than looped), so a launch costs about one
//    weight-load latency plus the merge.  W (the only HBM stream) is read
//    exactly once, with nontemporal loads; X and the norm weight are L2-hot.
//    The RMSNorm statistic comes precomputed from the kernel that produced X
//    (ss_in: fp32 partial sums over 16-column chunks), so no workgroup re-reads
//    whole X rows in a prologue.  Replaces the hipBLASLt M=64 GEMMs (measured
//    0.6 TB/s) plus the separate RMSNorm / SiLU / residual launches.
//
//  * attention decode (GQA), flash-decoding form — one workgroup (8 waves) per
//    (kv head, sequence): every lane issues the K and V loads of up to J keys
//    before the RoPE prologue, so the KV stream is one round trip; scores,
//    online softmax and P.V stay in registers, lanes/waves merge (m, l, acc).
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace swh {
// csrc/wide_gemm.hip: 1 = shape not eligible, else a SWH status
int wide_gemm(const void *x, const void *w, int64_t M, int64_t N, int64_t K, float eps, const float *ss_in,
              const void *bias, void *residual, int32_t silu, void *y, int64_t ldy, float *ss_out, void *workspace,
              int64_t workspace_bytes, int64_t counter_bytes, int32_t packed, hipStream_t stream);
int64_t wide_gemm_slab_bytes(int64_t M, int64_t N, int64_t K, int32_t silu);
bool wide_gemm_eligible(int64_t M, int64_t N, int64_t K, int32_t silu);
int wide_pack(const void *src, const void *norm_w, int64_t N, int64_t K, int32_t silu, void *dst, hipStream_t stream);
int wide_lm_sample(const void *x, const void *w, int64_t M, int64_t V, int64_t K, float eps, const float *ss_in,
                   const swh_sample_params &p, const uint64_t *rng, const int32_t *step, LmPart *part, int *pstride,
                   hipStream_t stream);
int frag_pack(const void *src, const void *norm_w, int64_t N, int64_t K, int32_t silu, void *dst, hipStream_t stream);

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = 64;  // rows per workgroup tile (M tile)
constexpr int64_t kCounterBytes = 1 << 16;  // split-K ticket counters (16384 tiles)

enum : int { EPI_PLAIN = 0, EPI_RESIDUAL = 1, EPI_SILU = 2 };

// Phase timestamps for tools/gemm_probe (a build with SWH_GEMM_TRACE_ON defined):
// wall clock (100 MHz) of wave 0 at each phase boundary, per workgroup.
#ifdef SWH_GEMM_TRACE_ON
__device__ unsigned long long *g_gemm_trace;
#define SWH_GEMM_TRACE(i)                                                                                      \
    if (threadIdx.x == 0 && g_gemm_trace)                                                                      \
    g_gemm_trace[((int64_t)(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + (i)] =        \
        wall_clock64()
#else
#define SWH_GEMM_TRACE(i)
#endif

// Workgroup barrier that waits for LDS traffic only: global loads issued
// before it stay in flight (the compiler's counted vmcnt waits cover uses).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ bf16x8 as_bf16x8(const uint4 &v) { return __builtin_bit_cast(bf16x8, v); }

// Normalised X: bf16(w * bf16(x * rstd)) for 8 consecutive k (Qwen2RMSNorm's
// two roundings), packed f32 math: 4 VALU per element.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t norm_pair(uint32_t xv, f32x2 w, float rs) {
    const f32x2 xf = {__uint_as_float(xv << 16), __uint_as_float(xv & 0xffff0000u)};
    const uint32_t tb = __builtin_bit_cast(uint32_t, __builtin_convertvector(xf * rs, bf16x2));
    const f32x2 tf = {__uint_as_float(tb << 16), __uint_as_float(tb & 0xffff0000u)};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(tf * w, bf16x2));
}
__device__ __forceinline__ uint4 norm_frag(const uint4 &xv, const float4 &w0, const float4 &w1, float rs) {
    return uint4{norm_pair(xv.x, f32x2{w0.x, w0.y}, rs), norm_pair(xv.y, f32x2{w0.z, w0.w}, rs),
                 norm_pair(xv.z, f32x2{w1.x, w1.y}, rs), norm_pair(xv.w, f32x2{w1.z, w1.w}, rs)};
}

__device__ __forceinline__ uint4 pack8(const float *v) {
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        o[k] = (uint32_t)f32_to_bf16_bits(v[2 * k]) | ((uint32_t)f32_to_bf16_bits(v[2 * k + 1]) << 16);
    return uint4{o[0], o[1], o[2], o[3]};
}


// LDS layout of the GEMM kernel (bytes; host and device compute it alike):
//   [0,256) rstd[64] | [256,272) flag | [512, ...) norm-weight slice (f32)
//   | RMSNorm partials [MR][K/64] f32 | the X image [MR][Kr*2+16 B] (LDS-DMA);
//     the merge slots [NW/2][NB][MR+4] f32 reuse the image, or follow it when
//     the workgroup loops over several column blocks (the image must persist).
struct GemmLds {
    int64_t nw_off, ss_off, body_off, xs_bytes, slots_off, total;
};
// nm: 0 = plain X, 1 = RMSNorm applied to the X image, 2 = rstd row scale in the epilogue
// cb: the tile's 16-column blocks; wn: column groups of waves (nw / wn waves split K in each)
__host__ __device__ inline GemmLds gemm_lds(int cb, int mr, int nw, int krmax, int K, int nm, bool persist,
                                            int wn = 1) {
    GemmLds L;
    L.nw_off = 512;
    L.ss_off = L.nw_off + (nm == 1 ? (int64_t)krmax * 4 : 0);  // norm weights as f32
    L.body_off = L.ss_off + (nm ? ((int64_t)mr * (K / 64) * 4 + 15) / 16 * 16 : 0);  // partials beside the DMA'd image
    L.xs_bytes = (int64_t)mr * (krmax * 2 + 16);
    const int wk = nw / wn;
    const int64_t slots = (int64_t)(wk + 1) * 16 * cb * (mr + 4) * 4;  // [WK + 1][NB][MR+4]
    L.slots_off = L.body_off + (persist ? L.xs_bytes : 0);
    int64_t end = L.body_off + L.xs_bytes;
    if (L.slots_off + slots > end) end = L.slots_off + slots;
    L.total = end;
    return L;
}

// Tile = MR (16 * MS) rows x NB (16 * CB) output columns x one K slice.
// A workgroup stages its X slice [MR rows x Kr] into LDS ONCE — every wave
// whole rows, lanes along the row (full-line 16-B loads), RMSNorm applied on
// the way in — then covers one column block, or several when the grid is
// smaller than the column blocks (the lm head loops, prefetching the next
// block's weights before merging the current one).  The NW waves split the
// slice's k-steps; each issues all weight loads of a round of U k-steps at
// once (fragment order) and takes its A fragments from the LDS image.  Waves
// merge through a fixed-order LDS tree.  Tiles are numbered so the M tiles of
// one column block land on one XCD (dispatch is round-robin over the 8 XCDs):
// their shared weight rows are fetched from HBM once and re-read from that
// XCD's L2.  S > 1: write-through (sc1) fp32 slabs, an agent-scope ticket, the
// last arriver sums the S slabs in fixed order (deterministic, placement-
// independent — MI355X_MICROARCH.md §Workgroup dispatch) and runs the epilogue.

#ifndef SWH_KU
#define SWH_KU 4  // weight-load round depth (k-steps per wave issued together)
#endif
#ifndef SWH_ROUND_PREFETCH
#define SWH_ROUND_PREFETCH 0  // all A reads of a full round before its MFMAs (A/B: tools/build_variant.py)
#endif
#ifndef SWH_W_NT
#define SWH_W_NT 0  // weight-stream loads with the non-temporal policy (A/B)
#endif
// one 16-B weight fragment (read once per launch)
__device__ __forceinline__ uint4 ld_w(const uint16_t *p) {
    if constexpr (SWH_W_NT) return ld_nt(reinterpret_cast<const uint4 *>(p));
    return *reinterpret_cast<const uint4 *>(p);
}
// the same with the non-temporal policy chosen per kernel: the gate/up tiles (fragment-order
// weights, whole 1 KB runs per load) gain from it (11.15 -> 10.7 us), while the projections
// whose weights the attention launch warms into the Infinity Cache (qkv, o, down) and the
// lm-head sampler lose (profiles/r5_wnt_ab.log, r5_gunt_ab.log)
template <bool NT>
__device__ __forceinline__ uint4 ld_wt(const uint16_t *p) {
    if constexpr (NT) return ld_nt(reinterpret_cast<const uint4 *>(p));
    return ld_w(p);
}
#ifndef SWH_GEMM_RING
#define SWH_GEMM_RING 0  // decode_gemm k-loop: refill each k-step's weight registers right after its MFMAs (A/B)
#endif
static_assert(!(SWH_GEMM_RING && SWH_ROUND_PREFETCH), "the ring refill lives in the per-k-step loop");
#ifndef SWH_SILU_ST16
#define SWH_SILU_ST16 1  // gate/up SiLU epilogue: 16-B row stores through a per-wave LDS tile (A/B)
#endif
#ifndef SWH_LM_RING
#define SWH_LM_RING 1  // lm-head tile loop: refill each weight register right after its MFMA (A/B)
#endif
#ifndef SWH_FLAT_MERGE
#define SWH_FLAT_MERGE 0  // one-barrier flat wave merge instead of the tree (A/B)
#endif

// KL: a K-class tag (0: K <= 1024, 1: longer) that only separates the rocprof
// names of otherwise identical instantiations (o_proj K 896 vs down_proj K 4864)
template <int CB, int MS, int NM, int EPI, bool BIAS, int MAXT, int KL = 0>
__global__ __launch_bounds__(MAXT) void decode_gemm_kernel(
    const uint16_t *__restrict__ x, const uint16_t *__restrict__ w, int M, int N, int K,
    const uint16_t *__restrict__ norm_w, float eps, const float *__restrict__ ss_in,
    const uint16_t *__restrict__ bias, uint16_t *__restrict__ res, float *__restrict__ ss_out,
    uint16_t *__restrict__ y, int ldy, float *__restrict__ slabs, int *__restrict__ counters, int persist,
    int wn, int fw) {
    // a wave computes NB = 16 CB columns; the WN column groups of NW / WN waves each
    // make a tile of NBT = WN NB columns (the waves of a group split K)
    constexpr int NB = 16 * CB, MR = 16 * MS, LDR = MR + 4;  // merge slots column-major: b128 parks
    constexpr int kU = SWH_KU;                                // k-steps whose loads are issued together
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, NT = blockDim.x, NW = NT >> 6;
    const int WN = wn, NBT = NB * WN, WK = NW / WN, cg = wid / WK, kw = wid - cg * WK;
    const int G8 = (EPI == EPI_SILU) ? CB * WN : NBT / 8;  // 8-column output groups per row
    const int S = gridDim.z, sidx = blockIdx.z;
    const int ncb = (EPI == EPI_SILU) ? N / (NBT / 2) : N / NBT;
    const int nmt = (M + MR - 1) / MR;
    // ---- tile of this workgroup
    int cb_first, cb_step, mt;
    if (persist) {  // gridDim.x % nmt == 0
        mt = blockIdx.x % nmt;
        cb_first = blockIdx.x / nmt;
        cb_step = gridDim.x / nmt;
        if (cb_first >= ncb) return;
    } else {        // the nmt M tiles of a column block on one XCD
        const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
        cb_first = (j / nmt) * 8 + xcd;
        mt = j % nmt;
        cb_step = ncb;
        if (cb_first >= ncb) return;
    }
    const int m0 = mt * MR;
    const int KS = K / 32, kb0 = (int)((int64_t)KS * sidx / S), kb1 = (int)((int64_t)KS * (sidx + 1) / S);
    const int Kr = (kb1 - kb0) * 32, k0 = kb0 * 32, RS = Kr * 2 + 16;
    const GemmLds L = gemm_lds(CB * WN, MR, NW, (KS + S - 1) / S * 32, K, NM, persist != 0, WN);
    float *rstd_s = reinterpret_cast<float *>(lds);
    int *flag_s = reinterpret_cast<int *>(lds + 256);
    float *nw_s = reinterpret_cast<float *>(lds + L.nw_off);
    unsigned char *xs = lds + L.body_off;
    float *ssp = reinterpret_cast<float *>(lds + L.ss_off);
    float *part = reinterpret_cast<float *>(lds + L.slots_off);
    const int rl = lane & 15, kq = (lane >> 4) * 8;
    SWH_GEMM_TRACE(0);

    // ---- (a) this wave's weights for the first column block (HBM, the long pole: first in the queue)
    const int ksw0 = kb0 + (kb1 - kb0) * kw / WK, ksw1 = kb0 + (kb1 - kb0) * (kw + 1) / WK;
    const uint16_t *wrow[CB];
    auto set_rows = [&](int n0) {
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            int n;
            if constexpr (EPI == EPI_SILU) {
                const int c = (cg * CB + j) * 8 + (rl & 7);
                n = (rl < 8) ? n0 + c : N + n0 + c;  // gate rows, then the matching up rows
            } else {
                n = n0 + (cg * CB + j) * 16 + rl;
            }
            // fw: the swh_frag_pack layout — 16-row group g, k-step ks, lane at ((g KS + ks) 64 + lane) 8
            // (SiLU: a 16-lane group is 8 gate + the 8 matching up rows = pack group (first gate row) / 8)
            const int64_t grp = (EPI == EPI_SILU) ? (n0 + (cg * CB + j) * 8) >> 3 : (n0 + (cg * CB + j) * 16) >> 4;
            wrow[j] = fw ? w + (grp * KS * 64 + lane) * 8 : w + (int64_t)n * K + kq;
        }
    };
    const int wstep = fw ? 512 : 32;  // elements between a lane's consecutive k-steps
    uint4 bv[kU][CB];
    auto issue = [&](int ks) {  // only this wave's k-steps: no duplicate loads
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (ks + u < ksw1) {
#pragma unroll
                for (int j = 0; j < CB; ++j)  // plain loads: the line's other half is the next k-step's load
                    bv[u][j] = ld_w(wrow[j] + (ks + u) * wstep);
            }
        }
    };
    auto col0 = [&](int cbk) { return cbk * (EPI == EPI_SILU ? NBT / 2 : NBT); };
    set_rows(col0(cb_first));
    issue(ksw0);
    // ---- (b) RMSNorm partial sums and the norm-weight slice (L2)
    const int nc = K / 64;
    // folded norm, one column block: the row statistic only scales the epilogue;
    // 8 lanes per row sum the row's chunk partials in registers (no LDS pass)
    const bool late_rstd = NM == 2 && !persist && ss_in && MR * 8 <= NT && nc <= 64;
    const bool use_ss = NM && ss_in && MR * nc <= 4 * NT && !late_rstd;
    float4 ssv[4];
    float4 ss8[8];
    uint4 nwv[2];
    if (late_rstd) {
        const int r = min(m0 + (tid >> 3), M - 1), sub = tid & 7;
        const float4 *row = reinterpret_cast<const float4 *>(ss_in + (int64_t)r * (K / 16));
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (sub + 8 * j < nc) ss8[j] = row[sub + 8 * j];
    }
    if constexpr (NM != 0) {
        if (use_ss) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int idx = min(tid + q * NT, MR * nc - 1);
                const int r = idx / nc, c = idx - r * nc;
                ssv[q] = reinterpret_cast<const float4 *>(ss_in + (int64_t)min(m0 + r, M - 1) * (K / 16))[c];
            }
        }
        if constexpr (NM == 1) {
#pragma unroll
            for (int q = 0; q < 2; ++q)
                nwv[q] = reinterpret_cast<const uint4 *>(norm_w + k0)[min(tid + q * NT, Kr / 8 - 1)];
        }
    }
    // epilogue operands of a single-block workgroup (L2): <= 2 per thread in every geometry
    const int ncol0 = col0(cb_first);
    uint4 pre_res[2], pre_bias[2];
    if constexpr (EPI == EPI_RESIDUAL || BIAS) {
        if (!persist) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int idx = min(tid + q * NT, MR * G8 - 1);
                const int r = idx / G8, gc = ncol0 + (idx - r * G8) * 8;
                if constexpr (EPI == EPI_RESIDUAL)
                    pre_res[q] = *reinterpret_cast<const uint4 *>(res + (int64_t)min(m0 + r, M - 1) * ldy + gc);
                if constexpr (BIAS) pre_bias[q] = *reinterpret_cast<const uint4 *>(bias + gc);
            }
        }
    }
    // ---- (c) X slice -> LDS image by LDS-DMA (no registers): each wave whole rows
    // wid, wid+NW, ...; one instruction = 64 lanes x 16 B = 1 KB of a row
    const int ppr = Kr / 8, jpl = (ppr + 63) >> 6;  // 16-B pieces per row, instructions per row
    for (int r = wid; r < MR; r += NW) {
        const uint16_t *src = x + (int64_t)min(m0 + r, M - 1) * K + k0;
        for (int j = 0; j < jpl; ++j) {
            const int c = lane + 64 * j;
            if (c < ppr)
                __builtin_amdgcn_global_load_lds(src + c * 8,
                                                 (__attribute__((address_space(3))) void *)(xs + r * RS + j * 1024),
                                                 16, 0, 0);
        }
    }
    // everything this workgroup streams is in flight; the image is usable once all of it landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    SWH_GEMM_TRACE(1);

    // ---- (d) row statistic and norm weights into LDS
    if (late_rstd) {  // read by the epilogue only, behind the merge barriers
        const int r = tid >> 3, sub = tid & 7;
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (sub + 8 * j < nc) v += ((ss8[j].x + ss8[j].y) + ss8[j].z) + ss8[j].w;
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        if (r < MR && sub == 0) rstd_s[r] = rsqrtf(v / (float)K + eps);
    } else if constexpr (NM != 0) {
        if (use_ss) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int idx = tid + q * NT;
                if (idx < MR * nc) ssp[idx] = ((ssv[q].x + ssv[q].y) + ssv[q].z) + ssv[q].w;
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (NM == 1 && tid + q * NT < Kr / 8) {
                float f[8];
                unpack16<SWH_BF16>(nwv[q], f);
                reinterpret_cast<float4 *>(nw_s)[2 * (tid + q * NT)] = float4{f[0], f[1], f[2], f[3]};
                reinterpret_cast<float4 *>(nw_s)[2 * (tid + q * NT) + 1] = float4{f[4], f[5], f[6], f[7]};
            }
        lds_barrier();
        if (use_ss) {
            if (tid < MR) {
                float ssum = 0.f;
                for (int c = 0; c < nc; ++c) ssum += ssp[tid * nc + c];
                rstd_s[tid] = rsqrtf(ssum / (float)K + eps);
            }
        } else {
            // whole-row pass over X in global memory, one wave per row (coalesced)
            const int nv = K / 8;
            for (int r = wid; r < MR; r += NW) {
                const uint4 *xr = reinterpret_cast<const uint4 *>(x + (int64_t)min(m0 + r, M - 1) * K);
                float ss = 0.f;
                for (int v = lane; v < nv; v += 64) {
                    float a[8];
                    unpack16<SWH_BF16>(xr[v], a);
#pragma unroll
                    for (int k = 0; k < 8; ++k) ss = fmaf(a[k], a[k], ss);
                }
                ss = wave_sum(ss);
                if (lane == 0) rstd_s[r] = rsqrtf(ss / (float)K + eps);
            }
        }
        lds_barrier();
    }
    SWH_GEMM_TRACE(2);

    // ---- (e) the X image normalised in place
    if constexpr (NM == 1) {
        int r = tid / ppr, c = tid - r * ppr;
        const int rstep = NT / ppr, cstep = NT - rstep * ppr;
        for (; r < MR;) {
            uint4 *pv = reinterpret_cast<uint4 *>(xs + r * RS + c * 16);
            const float4 *wv = reinterpret_cast<const float4 *>(nw_s) + 2 * c;
            *pv = norm_frag(*pv, wv[0], wv[1], rstd_s[r]);
            r += rstep;
            c += cstep;
            if (c >= ppr) {
                c -= ppr;
                ++r;
            }
        }
        lds_barrier();
    }
    SWH_GEMM_TRACE(3);

    // ---- (f) column blocks
    auto slot = [&](int s, int r, int c) -> float & { return part[(s * NBT + c) * LDR + r]; };
    const int F = WK;  // the merged slot
    for (int cbk = cb_first; cbk < ncb; cbk += cb_step) {
        const int n0 = col0(cbk);
        f32x4 acc[MS][CB];
#pragma unroll
        for (int i = 0; i < MS; ++i)
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        const unsigned char *xrow = xs + rl * RS + kq * 2;
        for (int ks = ksw0; ks < ksw1; ks += kU) {
            if (!SWH_GEMM_RING && ks != ksw0) issue(ks);
            const unsigned char *xk = xrow + (ks - kb0) * 64;
            if (SWH_ROUND_PREFETCH && ks + kU <= ksw1) {  // a full round: every A fragment read in flight first
                uint4 a[kU][MS];
#pragma unroll
                for (int u = 0; u < kU; ++u)
#pragma unroll
                    for (int i = 0; i < MS; ++i) a[u][i] = *reinterpret_cast<const uint4 *>(xk + i * 16 * RS + u * 64);
#pragma unroll
                for (int u = 0; u < kU; ++u)
#pragma unroll
                    for (int i = 0; i < MS; ++i)
#pragma unroll
                        for (int j = 0; j < CB; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[u][i]), as_bf16x8(bv[u][j]),
                                                                                acc[i][j], 0, 0, 0);
            } else {
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    if (ks + u >= ksw1) break;
                    uint4 a[MS];
#pragma unroll
                    for (int i = 0; i < MS; ++i) a[i] = *reinterpret_cast<const uint4 *>(xk + i * 16 * RS + u * 64);
#pragma unroll
                    for (int i = 0; i < MS; ++i)
#pragma unroll
                        for (int j = 0; j < CB; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[i]), as_bf16x8(bv[u][j]),
                                                                                acc[i][j], 0, 0, 0);
                    if (SWH_GEMM_RING && ks + kU + u < ksw1) {
                        // ring refill: k-step ks + u's registers take k-step ks + kU + u as soon as
                        // its MFMAs have read them, so kU k-steps stay in flight per wave
#pragma unroll
                        for (int j = 0; j < CB; ++j)
                            bv[u][j] = ld_w(wrow[j] + (ks + kU + u) * wstep);
                    }
                }
            }
        }
        // the next column block's first weight round overlaps this block's merge
        if (cbk + cb_step < ncb) {
            set_rows(col0(cbk + cb_step));
            issue(ksw0);
        }
        SWH_GEMM_TRACE(4);

#if SWH_FLAT_MERGE
        // ---- merge the K-splitting waves: every wave parks its partial in its own slot,
        // one barrier, then each output element sums the WK slots in fixed order into
        // slot F = WK (two barriers instead of a log2(WK)-level tree)
        if (!persist) lds_barrier();  // the slots reuse the X image
        // C layout: lane holds rows 16 i + 4 g .. +3 of column 16 j + rl -> one 16-B store each
#pragma unroll
        for (int i = 0; i < MS; ++i)
#pragma unroll
            for (int j = 0; j < CB; ++j)
                *reinterpret_cast<f32x4 *>(&slot(kw, i * 16 + (lane >> 4) * 4, (cg * CB + j) * 16 + rl)) = acc[i][j];
        lds_barrier();
        for (int idx = tid; idx < MR * NBT; idx += NT) {
            const int c = idx / MR, r = idx - c * MR;  // r fastest: consecutive banks
            float v = part[c * LDR + r];
            for (int q = 1; q < WK; ++q) v += part[(q * NBT + c) * LDR + r];
            part[(F * NBT + c) * LDR + r] = v;
        }
        lds_barrier();
#else
        // ---- merge the NW waves: fixed-order tree through the LDS slots -> slot F
        if (!persist) lds_barrier();  // the slots reuse the X image
        auto park = [&](int s) {
#pragma unroll
            for (int i = 0; i < MS; ++i)
#pragma unroll
                for (int j = 0; j < CB; ++j)
                    *reinterpret_cast<f32x4 *>(&slot(s, i * 16 + (lane >> 4) * 4, (cg * CB + j) * 16 + rl)) = acc[i][j];
        };
        for (int h = WK >> 1; h >= 1; h >>= 1) {
            if (kw >= h && kw < 2 * h) park(kw - h);
            lds_barrier();
            if (kw < h) {
#pragma unroll
                for (int i = 0; i < MS; ++i)
#pragma unroll
                    for (int j = 0; j < CB; ++j)
                        acc[i][j] += *reinterpret_cast<const f32x4 *>(
                            &slot(kw, i * 16 + (lane >> 4) * 4, (cg * CB + j) * 16 + rl));
            }
            lds_barrier();
        }
        if (kw == 0) park(F);
        lds_barrier();
#endif
        SWH_GEMM_TRACE(5);

        // ---- cross-workgroup split-K: publish, ticket, last arriver reduces
        if (S > 1) {
            const int blk = mt * ncb + cbk;
            float *my = slabs + ((int64_t)blk * S + sidx) * (MR * NBT);
            for (int idx = tid; idx < MR * NBT; idx += NT)
                __hip_atomic_store(my + idx, slot(F, idx / NBT, idx % NBT), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                const int t = __hip_atomic_fetch_add(counters + blk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                flag_s[0] = (t == S - 1);
            }
            __syncthreads();
            if (!flag_s[0]) return;  // S > 1 never loops over column blocks
            const float *base = slabs + (int64_t)blk * S * (MR * NBT);
            for (int idx = tid; idx < MR * NBT; idx += NT) {
                float v = 0.f;
                for (int q = 0; q < S; ++q)
                    v += __hip_atomic_load(base + (int64_t)q * MR * NBT + idx, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                slot(F, idx / NBT, idx % NBT) = v;
            }
            if (tid == 0) __hip_atomic_store(counters + blk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
        }

        // ---- epilogue, 8 output columns (16 B) per thread
        if constexpr (EPI == EPI_SILU) {
            for (int idx = tid; idx < MR * G8; idx += NT) {
                const int r = idx / G8, jb = idx - r * G8;
                const int gr = m0 + r;
                if (gr >= M) continue;
                float o[8];
                const float sc = (NM == 2) ? rstd_s[r] : 1.f;  // folded RMSNorm: y = rstd * (x W'^T)
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) {
                    const float g = round_bf16(slot(F, r, jb * 16 + cc) * sc);
                    const float u = round_bf16(slot(F, r, jb * 16 + 8 + cc) * sc);
                    o[cc] = round_bf16(g / (1.f + expf(-g))) * u;
                }
                *reinterpret_cast<uint4 *>(y + (int64_t)gr * ldy + n0 + jb * 8) = pack8(o);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int idx = tid + q * NT;
                if (idx >= MR * G8) break;
                const int r = idx / G8, c8 = (idx - r * G8) * 8;
                const int gr = m0 + r, gc = n0 + c8;
                if (gr >= M) continue;
                float v[8];
                const float sc = (NM == 2) ? rstd_s[r] : 1.f;  // folded RMSNorm: y = rstd * (x W'^T)
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) v[cc] = slot(F, r, c8 + cc) * sc;
                if constexpr (BIAS) {
                    float b[8];
                    unpack16<SWH_BF16>(persist ? *reinterpret_cast<const uint4 *>(bias + gc) : pre_bias[q], b);
#pragma unroll
                    for (int cc = 0; cc < 8; ++cc) v[cc] += b[cc];
                }
                if constexpr (EPI == EPI_RESIDUAL) {
                    uint4 *sp = reinterpret_cast<uint4 *>(res + (int64_t)gr * ldy + gc);
                    float sres[8];
                    unpack16<SWH_BF16>(persist ? *sp : pre_res[q], sres);
#pragma unroll
                    for (int cc = 0; cc < 8; ++cc) {
                        sres[cc] = round_bf16(sres[cc] + round_bf16(v[cc]));
                        slot(F, r, c8 + cc) = sres[cc];
                    }
                    *sp = pack8(sres);
                } else {
                    *reinterpret_cast<uint4 *>(y + (int64_t)gr * ldy + gc) = pack8(v);
                }
            }
            if constexpr (EPI == EPI_RESIDUAL) {
                if (ss_out) {  // partial sums of squares of the new rows, per 16-column chunk
                    __syncthreads();
                    for (int idx = tid; idx < MR * CB * WN; idx += NT) {
                        const int r = idx / (CB * WN), j = idx - r * (CB * WN);
                        if (m0 + r >= M) continue;
                        float ss = 0.f;
#pragma unroll
                        for (int cc = 0; cc < 16; ++cc) ss = fmaf(slot(F, r, j * 16 + cc), slot(F, r, j * 16 + cc), ss);
                        ss_out[(int64_t)(m0 + r) * (N / 16) + n0 / 16 + j] = ss;
                    }
                }
            }
        }
        if (persist) __syncthreads();  // slot 0 is rewritten by the next block
    }
    SWH_GEMM_TRACE(6);
}

// Infinity Cache warm-up job: a device range read (and discarded) by warm-up workgroups
struct L3Job {
    const uint4 *p;
    int64_t n16;       // 16-B units
    int64_t reserved;  // 0
};
constexpr int kL3MaxJobs = 8;

// warm-up workgroup p of npf (NT threads): a contiguous share of the jobs' bytes,
// 8 x 16-B loads in flight per thread, XOR-ed into a word stored only if it
// equals a magic constant
template <int NT>
__device__ __forceinline__ void l3_warm_share(const L3Job *__restrict__ jobs, int njobs, int p, int npf,
                                              uint32_t *__restrict__ sink) {
    const int tid = threadIdx.x;
    int64_t tot = 0;
    for (int j = 0; j < njobs; ++j) tot += jobs[j].n16;
    const int64_t share = (tot + npf - 1) / npf, lo = (int64_t)p * share, hi = min(tot, lo + share);
    uint32_t acc = 0;
    auto sweep = [&](const uint4 *src, int64_t a, int64_t e) {
        for (int64_t i = a + tid; i < e; i += 8 * NT) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t q = i + u * NT;
                v[u] = q < e ? src[q] : uint4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    };
    int64_t base = 0;
    for (int j = 0; j < njobs; ++j) {
        const int64_t n = jobs[j].n16;
        sweep(jobs[j].p, max(lo - base, (int64_t)0), min(hi - base, n));
        base += n;
    }
    if (acc == 0x9e3779b9u) sink[(int64_t)p * NT + tid] = acc;
}

// ---------------------------------------------------------------------------
// Register-streamed short-K projection (decode qkv and o_proj at K <= 2048:
// 16 MS-row x 16-column tiles over the full K, no K split): decode_gemm_kernel
// <1, MS, NM, EPI, BIAS> with the X slice read as MFMA A fragments straight
// into registers beside the weight fragments.  A wave's A operand is X[MR rows,
// its own k-steps], which no other wave reads, so the LDS image — and its
// landing wait (vmcnt(0)) before the first MFMA — goes: every k-step of the
// wave is issued at once (KW of them) and the MFMAs consume them in arrival
// order.  Same k-step split, wave order, merge tree, row statistic and
// epilogues as decode_gemm_kernel, so the result is bit-identical.  At long K
// (down_proj, K 4864) the fragment-order X loads (64 B of a row per lane group,
// twice the lines of the image's whole-row loads) cost more than the landing
// wait saves (11.4 -> 12.4 us), so it serves K <= 2048 only.
// ---------------------------------------------------------------------------
template <int KW, int MS, int NM, int EPI, bool BIAS, int KL>
__global__ __launch_bounds__(512) void xstream_gemm_kernel(const uint16_t *__restrict__ x,
                                                           const uint16_t *__restrict__ w, int M, int N, int K,
                                                           float eps, const float *__restrict__ ss_in,
                                                           const uint16_t *__restrict__ bias,
                                                           uint16_t *__restrict__ res, float *__restrict__ ss_out,
                                                           uint16_t *__restrict__ y, int ldy, int fw, int xf) {
    static_assert(EPI != EPI_SILU && NM != 1, "plain / residual epilogues, folded or no norm");
    constexpr int NW = 8, NT = 512, MR = 16 * MS, NB = 16, LDR = MR + 4, G8 = NB / 8, F = NW;
    __shared__ __attribute__((aligned(16))) float part[(NW + 1) * NB * LDR];
    __shared__ float rstd_s[MR];
    const int tid = threadIdx.x, lane = tid & 63, kw = tid >> 6;
    const int ncb = N / NB, nmt = (M + MR - 1) / MR;
    const int xcd = blockIdx.x & 7, jj = blockIdx.x >> 3;  // the nmt M tiles of a column block on one XCD
    const int cbk = (jj / nmt) * 8 + xcd, mt = jj % nmt;
    if (cbk >= ncb) return;
    const int m0 = mt * MR, n0 = cbk * NB;
    const int KS = K / 32, ksw0 = KS * kw / NW, ksw1 = KS * (kw + 1) / NW;
    const int rl = lane & 15, kq = (lane >> 4) * 8;
    SWH_GEMM_TRACE(0);
    // epilogue operands and the row statistic's partials (oldest in the queue)
    uint4 pre_ep;
    {
        const int idx = min(tid, MR * G8 - 1);
        const int r = idx / G8, gc = n0 + (idx - r * G8) * 8;
        if constexpr (EPI == EPI_RESIDUAL)
            pre_ep = *reinterpret_cast<const uint4 *>(res + (int64_t)min(m0 + r, M - 1) * ldy + gc);
        else if constexpr (BIAS)
            pre_ep = *reinterpret_cast<const uint4 *>(bias + gc);
    }
    const int nc = K / 64;
    float4 ss8[8];
    if constexpr (NM == 2) {
        const int r = min(m0 + (tid >> 3), M - 1), sub = tid & 7;
        const float4 *row = reinterpret_cast<const float4 *>(ss_in + (int64_t)r * (K / 16));
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (sub + 8 * j < nc) ss8[j] = row[sub + 8 * j];
    }
    // fw: the swh_frag_pack layout (one contiguous 1 KB per wave and k-step)
    const uint16_t *wr = fw ? w + ((int64_t)(n0 >> 4) * KS * 64 + lane) * 8 : w + (int64_t)(n0 + rl) * K + kq;
    const int wstep = fw ? 512 : 32;
    // xf: X itself in the fragment order (16-row groups; written so by the SiLU tile
    // epilogue, M % 16 == 0): one contiguous 1 KB run per A-fragment load as well
    const uint16_t *xr[MS];
#pragma unroll
    for (int i = 0; i < MS; ++i)
        xr[i] = xf ? x + ((int64_t)((m0 >> 4) + i) * KS * 64 + lane) * 8
                   : x + (int64_t)min(m0 + i * 16 + rl, M - 1) * K + kq;
    const int xstep = xf ? 512 : 32;
    uint4 xa[KW][MS], bv[KW];
#pragma unroll
    for (int u = 0; u < KW; ++u) {
        const int ks = min(ksw0 + u, ksw1 - 1);  // past the wave's range: a repeated, unused load (no branch)
        bv[u] = ld_w(wr + ks * wstep);
#pragma unroll
        for (int i = 0; i < MS; ++i) xa[u][i] = *reinterpret_cast<const uint4 *>(xr[i] + ks * xstep);
    }
    SWH_GEMM_TRACE(1);
    if constexpr (NM == 2) {  // read by the epilogue only, behind the merge barriers
        const int r = tid >> 3, sub = tid & 7;
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (sub + 8 * j < nc) v += ((ss8[j].x + ss8[j].y) + ss8[j].z) + ss8[j].w;
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        if (r < MR && sub == 0) rstd_s[r] = rsqrtf(v / (float)K + eps);
    }
    f32x4 acc[MS];
#pragma unroll
    for (int i = 0; i < MS; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < KW; ++u)
        if (ksw0 + u < ksw1) {
#pragma unroll
            for (int i = 0; i < MS; ++i)
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xa[u][i]), as_bf16x8(bv[u]), acc[i], 0, 0, 0);
        }
    SWH_GEMM_TRACE(4);
    // merge the 8 waves: decode_gemm_kernel's fixed-order tree -> slot F
    auto slot = [&](int s, int r, int c) -> float & { return part[(s * NB + c) * LDR + r]; };
    auto park = [&](int s) {
#pragma unroll
        for (int i = 0; i < MS; ++i) *reinterpret_cast<f32x4 *>(&slot(s, i * 16 + (lane >> 4) * 4, rl)) = acc[i];
    };
    for (int h = NW >> 1; h >= 1; h >>= 1) {
        if (kw >= h && kw < 2 * h) park(kw - h);
        lds_barrier();
        if (kw < h) {
#pragma unroll
            for (int i = 0; i < MS; ++i) acc[i] += *reinterpret_cast<const f32x4 *>(&slot(kw, i * 16 + (lane >> 4) * 4, rl));
        }
        lds_barrier();
    }
    if (kw == 0) park(F);
    lds_barrier();
    SWH_GEMM_TRACE(5);
    // epilogue, 8 output columns (16 B) per thread
    if (tid < MR * G8) {
        const int r = tid / G8, c8 = (tid - r * G8) * 8;
        const int gr = m0 + r, gc = n0 + c8;
        if (gr < M) {
            float v[8];
            const float sc = (NM == 2) ? rstd_s[r] : 1.f;  // folded RMSNorm: y = rstd * (x W'^T)
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) v[cc] = slot(F, r, c8 + cc) * sc;
            if constexpr (EPI == EPI_RESIDUAL) {
                float sres[8];
                unpack16<SWH_BF16>(pre_ep, sres);
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) {
                    sres[cc] = round_bf16(sres[cc] + round_bf16(v[cc]));
                    slot(F, r, c8 + cc) = sres[cc];
                }
                *reinterpret_cast<uint4 *>(res + (int64_t)gr * ldy + gc) = pack8(sres);
            } else {
                if constexpr (BIAS) {
                    float b[8];
                    unpack16<SWH_BF16>(pre_ep, b);
#pragma unroll
                    for (int cc = 0; cc < 8; ++cc) v[cc] += b[cc];
                }
                *reinterpret_cast<uint4 *>(y + (int64_t)gr * ldy + gc) = pack8(v);
            }
        }
    }
    if constexpr (EPI == EPI_RESIDUAL) {
        if (ss_out) {  // partial sums of squares of the new rows over this 16-column chunk
            __syncthreads();
            if (tid < MR && m0 + tid < M) {
                float ss = 0.f;
#pragma unroll
                for (int cc = 0; cc < 16; ++cc) ss = fmaf(slot(F, tid, cc), slot(F, tid, cc), ss);
                ss_out[(int64_t)(m0 + tid) * (N / 16) + n0 / 16] = ss;
            }
        }
    }
    SWH_GEMM_TRACE(6);
}

// ---------------------------------------------------------------------------
// Tile kernel (many 16-column tiles, K <= 1024: the lm head, gate/up):
// persistent workgroups, one per CU (per M tile); the X image [64 x K] is
// staged (and normalised) once, then every wave owns whole 16-column tiles
// over the full K — all K/32 weight loads of a tile in flight at once, the
// next tile's issued as soon as the MFMAs have consumed the current one, no
// cross-wave merge.  Tile t goes to workgroup t % wgs, so every CU gets work
// even when tiles are few.  Epilogues: plain (+ bias), SiLU gate (a tile is
// 8 gate + 8 up columns), or the fused sampler.
// ---------------------------------------------------------------------------
constexpr int kLmMaxKS = 32;  // K <= 1024

// Fused sampler (SAMPLE): instead of storing logits, each wave folds its
// tiles into per-row Gumbel-max bests (the unfiltered swh_sample_step: EOS
// suppression, temperature, greedy) and writes one partial per row; the
// Philox block at counter {col, row >> 2} holds the four rows a lane owns.
struct LmSample {
    swh_sample_params p;
    const uint64_t *rng;
    const int32_t *step;
    LmPart *part;  // [M][pstride]
    int pstride;
    int fw = 0;    // weights in the swh_frag_pack layout (tile t = 16-row group t)
    int yf = 0;    // SiLU output in the fragment order down_proj's A operand reads (N % 32 == 0)
    float2 *lpart = nullptr;  // log-prob variants: [M][pstride] (max, sum e^(z - max)) of the processed scores
};

// Reductions over one 16-lane DPP row (the 16 column lanes of a C-layout row group):
// quad_perm xor 1, quad_perm xor 2, row_half_mirror, row_mirror.  Every stage pairs
// lanes symmetrically, so all 16 lanes end with bit-identical values.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_max(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    return fmaxf(v, dpp_f<0x140>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    return v + dpp_f<0x140>(v);
}

// KSC: K / 32 at compile time (0 = read from K): with a constant trip count the
// compiler pipelines the A-fragment LDS reads across k-steps and waits on each
// weight load in turn (vmcnt(k)), instead of one LDS round trip per MFMA
// behind a wait for the whole tile (the lm head ran 5.6 us of MFMA per tile).
// RD: weight-ring depth in k-steps (0: the whole tile, KSC).  RD = KSC / 2 holds half a
// tile per wave (the k-steps ks + RD of the same tile, then the next tile's, refill each
// register), which fits three 12-wave... waves per SIMD: 768-thread workgroups.
// SAMPLE: 0 a plain GEMM epilogue, 1 the fused sampler, 2 the fused sampler with the
// temperature division (T != 1); 3 / 4: 1 / 2 plus the log-normaliser of the processed
// scores (the drawn token's log-prob, swh_lm_head_sample_logp): per tile and row a
// 16-lane max and sum of e^(z - max), folded into one running (max, sum) per lane —
// lane rl owns row 16 (rl >> 2) + 4 g + (rl & 3) — so the state costs two registers
template <int NM, int EPI, bool BIAS, int SAMPLE, int KSC, int RD = 0>
__global__ __launch_bounds__(RD ? 768 : 512) void lm_head_kernel(const uint16_t *__restrict__ x, const uint16_t *__restrict__ w,
                                                      int M, int N, int K, const uint16_t *__restrict__ norm_w,
                                                      float eps, const float *__restrict__ ss_in,
                                                      const uint16_t *__restrict__ bias, uint16_t *__restrict__ y,
                                                      int ldy, LmSample smp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, NT = blockDim.x, NW = NT >> 6;
    const int rl = lane & 15, kq = (lane >> 4) * 8, g = lane >> 4;
    const int nmt = (M + 63) / 64, mt = blockIdx.x % nmt, m0 = mt * 64;
    const int wgs = gridDim.x / nmt, wg = blockIdx.x / nmt;
    constexpr int KSA = KSC ? KSC : kLmMaxKS;  // register array extent
    const int ntile = (EPI == EPI_SILU) ? N / 8 : N / 16, KS = KSC ? KSC : K / 32, RS = K * 2 + 16;
    const GemmLds L = gemm_lds(1, 64, NW, K, K, NM, false);
    float *rstd_s = reinterpret_cast<float *>(lds);
    float *nw_s = reinterpret_cast<float *>(lds + L.nw_off);
    float *ssp = reinterpret_cast<float *>(lds + L.ss_off);
    unsigned char *xs = lds + L.body_off;
    const int tstep = wgs * NW;
    int t = wg + wgs * wid;  // tile t -> workgroup t % wgs
    SWH_GEMM_TRACE(0);

    static_assert(RD == 0 || (KSC != 0 && KSC % RD == 0 && 2 * RD == KSC), "RD: half of a compile-time tile");
    constexpr int KR = RD ? RD : KSA;  // weight registers per lane
    uint4 bv[KR];
    auto wrow_of = [&](int tile) -> int64_t {
        if constexpr (EPI == EPI_SILU) return (rl < 8) ? tile * 8 + rl : N + tile * 8 + rl - 8;  // gate, then up
        return (int64_t)tile * 16 + rl;
    };
    // fw 1: tile t's fragments for k-step ks at ((t KS + ks) 64 + lane) 8 (one 1 KB run per load)
    const int64_t wst = smp.fw ? 512 : 32;
    auto wbase = [&](int tile) -> const uint16_t * {
        return smp.fw ? w + ((int64_t)tile * KS * 64 + lane) * 8 : w + wrow_of(tile) * K + kq;
    };
    auto issue = [&](int tile) {
        const uint16_t *wr = wbase(tile);
#pragma unroll
        for (int ks = 0; ks < KR; ++ks)
            if (KSC || ks < KS) bv[ks] = ld_wt<EPI == EPI_SILU>(wr + ks * wst);
    };
    if (t < ntile) issue(t);  // the weight stream first
    // RMSNorm partials and norm weights (L2), then the X image by LDS-DMA
    const int nc = K / 64;
    // folded norm: 8 lanes per row sum the row's chunk partials in registers and the
    // row statistic is in LDS by the image barrier (no LDS pass, no extra barrier)
    const bool reg_rstd = NM == 2 && ss_in && 64 * 8 <= NT && nc <= 64;
    const bool use_ss = NM && ss_in && 64 * nc <= 4 * NT && !reg_rstd;
    float4 ssv[4];
    float4 ss8[8];
    uint4 nwv[2];
    if (reg_rstd) {
        const int r = min(m0 + (tid >> 3), M - 1), sub = tid & 7;
        const float4 *row = reinterpret_cast<const float4 *>(ss_in + (int64_t)r * (K / 16));
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (sub + 8 * j < nc) ss8[j] = row[sub + 8 * j];
    }
    if constexpr (NM != 0) {
        if (use_ss) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int idx = min(tid + q * NT, 64 * nc - 1);
                const int r = idx / nc, c = idx - r * nc;
                ssv[q] = reinterpret_cast<const float4 *>(ss_in + (int64_t)min(m0 + r, M - 1) * (K / 16))[c];
            }
        }
        if constexpr (NM == 1) {
#pragma unroll
            for (int q = 0; q < 2; ++q) nwv[q] = reinterpret_cast<const uint4 *>(norm_w)[min(tid + q * NT, K / 8 - 1)];
        }
    }
    const int ppr = K / 8, jpl = (ppr + 63) >> 6;
    for (int r = wid; r < 64; r += NW) {
        const uint16_t *src = x + (int64_t)min(m0 + r, M - 1) * K;
        for (int j = 0; j < jpl; ++j) {
            const int c = lane + 64 * j;
            if (c < ppr)
                __builtin_amdgcn_global_load_lds(src + c * 8,
                                                 (__attribute__((address_space(3))) void *)(xs + r * RS + j * 1024),
                                                 16, 0, 0);
        }
    }
    if constexpr (NM != 0) {
        if (use_ss) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int idx = tid + q * NT;
                if (idx < 64 * nc) ssp[idx] = ((ssv[q].x + ssv[q].y) + ssv[q].z) + ssv[q].w;
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (NM == 1 && tid + q * NT < K / 8) {
                float f[8];
                unpack16<SWH_BF16>(nwv[q], f);
                reinterpret_cast<float4 *>(nw_s)[2 * (tid + q * NT)] = float4{f[0], f[1], f[2], f[3]};
                reinterpret_cast<float4 *>(nw_s)[2 * (tid + q * NT) + 1] = float4{f[4], f[5], f[6], f[7]};
            }
    }
    SWH_GEMM_TRACE(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // image (and this wave's first tile) landed
    if (reg_rstd) {
        const int r = tid >> 3, sub = tid & 7;
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (sub + 8 * j < nc) v += ((ss8[j].x + ss8[j].y) + ss8[j].z) + ss8[j].w;
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        if (r < 64 && sub == 0) rstd_s[r] = rsqrtf(v / (float)K + eps);
    }
    lds_barrier();
    SWH_GEMM_TRACE(2);
    if (NM != 0 && !reg_rstd) {
        if (tid < 64) {
            float ssum = 0.f;
            if (use_ss) {
                for (int c = 0; c < nc; ++c) ssum += ssp[tid * nc + c];
            } else {  // from the (raw) image: the whole row is here
                for (int c = 0; c < ppr; ++c) {
                    float a[8];
                    unpack16<SWH_BF16>(*reinterpret_cast<const uint4 *>(xs + tid * RS + c * 16), a);
#pragma unroll
                    for (int k = 0; k < 8; ++k) ssum = fmaf(a[k], a[k], ssum);
                }
            }
            rstd_s[tid] = rsqrtf(ssum / (float)K + eps);
        }
        lds_barrier();
    }
    SWH_GEMM_TRACE(3);
    float rsr[4][4];  // folded RMSNorm (NM 2): the row scale of each accumulator row
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) rsr[i][e] = (NM == 2) ? rstd_s[i * 16 + 4 * g + e] : 1.f;
    if constexpr (NM == 1) {
        int r = tid / ppr, c = tid - r * ppr;
        const int rstep = NT / ppr, cstep = NT - rstep * ppr;
        while (r < 64) {
            uint4 *pv = reinterpret_cast<uint4 *>(xs + r * RS + c * 16);
            const float4 *wv = reinterpret_cast<const float4 *>(nw_s) + 2 * c;
            *pv = norm_frag(*pv, wv[0], wv[1], rstd_s[r]);
            r += rstep;
            c += cstep;
            if (c >= ppr) {
                c -= ppr;
                ++r;
            }
        }
        lds_barrier();
    }
    // sampler state: per lane the best (key, column) of its 16 rows 16 i + 4 g + e
    constexpr bool TDIV = SAMPLE == 2 || SAMPLE == 4, LOGP = SAMPLE >= 3;
    float bk[4][4];
    int32_t bi[4][4];
    uint32_t k0 = 0, k1 = 0, clo = 0, chi = 0;
    bool suppress = false;
    float temp = 1.f;
    float lm_run = kNegInf, ls_run = 0.f;  // LOGP: the owned row's running (max, sum e^(z - max))
    if constexpr (SAMPLE) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                bk[i][e] = kNegInf;
                bi[i][e] = 0x7fffffff;
            }
        const int32_t step = *smp.step;
        const uint64_t seed = smp.rng[0], ctr = smp.rng[1] + (uint64_t)step;
        k0 = (uint32_t)seed;
        k1 = (uint32_t)(seed >> 32);
        clo = (uint32_t)ctr;
        chi = (uint32_t)(ctr >> 32);
        suppress = step < smp.p.min_new_tokens;
        temp = (!smp.p.greedy && smp.p.temperature != 1.0f) ? smp.p.temperature : 1.f;
    }
    for (; t < ntile; t += tstep) {
        f32x4 acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        const unsigned char *xrow = xs + rl * RS + kq * 2;
        // ring refill: k-step ks's weight register takes the next tile's fragment as
        // soon as its MFMA has read it, so a wave always has KS loads in flight
        const bool ring = SWH_LM_RING && KSC != 0 && t + tstep < ntile;
        const uint16_t *wnext = wbase(ring ? t + tstep : t);
        const uint16_t *wcur = wbase(t);
        if constexpr (KSC != 0) {
            // A fragments double-buffered one k-step ahead (2 and 3 ahead measured no faster
            // for gate/up: 11.24 / 11.38-11.42 against 11.15-11.21 us, profiles/r5_gu_apf_ab.log);
            // the scheduling barrier keeps the compiler from hoisting every read
            constexpr int APF = 1, AR = APF + 1;
            uint4 a[AR][4];
#pragma unroll
            for (int p = 0; p < APF; ++p)
#pragma unroll
                for (int i = 0; i < 4; ++i) a[p][i] = *reinterpret_cast<const uint4 *>(xrow + i * 16 * RS + p * 64);
#pragma unroll
            for (int ks = 0; ks < KSC; ++ks) {
                if (ks + APF < KSC) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        a[(ks + APF) % AR][i] = *reinterpret_cast<const uint4 *>(xrow + i * 16 * RS + (ks + APF) * 64);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[ks % AR][i]), as_bf16x8(bv[ks % KR]),
                                                                    acc[i], 0, 0, 0);
                if constexpr (RD != 0) {  // half-tile ring: this tile's second half, then the next tile's first
                    if (ks + KR < KSC) bv[ks % KR] = ld_wt<EPI == EPI_SILU>(wcur + (ks + KR) * wst);
                    else if (ring) bv[ks % KR] = ld_wt<EPI == EPI_SILU>(wnext + (ks + KR - KSC) * wst);
                } else if (ring) {
                    bv[ks] = ld_wt<EPI == EPI_SILU>(wnext + ks * wst);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < KSA; ++ks) {
                if (ks < KS) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint4 a = *reinterpret_cast<const uint4 *>(xrow + i * 16 * RS + ks * 64);
                        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a), as_bf16x8(bv[ks]), acc[i], 0, 0, 0);
                    }
                }
            }
        }
        if (!ring && t + tstep < ntile) issue(t + tstep);
        SWH_GEMM_TRACE(4);
        if constexpr (SAMPLE) {
            const int col = t * 16 + rl;
            // EOS suppression as an added -inf (x + 0 = x), not a branch per element; the
            // temperature division only in the SAMPLE == 2 instantiation (T != 1): as a select,
            // the IEEE division ran on every element at T = 1 too
            float mask_add = 0.f;
            if (suppress) {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (e < smp.p.n_eos && col == smp.p.eos_ids[e]) mask_add = kNegInf;
            }
            float own_m = kNegInf, own_s = 0.f;  // LOGP: this tile's (max, sum) of the lane's owned row
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                U4 rw{0u, 0u, 0u, 0u};
                if (!smp.p.greedy) rw = philox4x32_10(U4{(uint32_t)col, (uint32_t)((m0 >> 2) + 4 * i + g), clo, chi}, k0, k1);
                const uint32_t wd[4] = {rw.x, rw.y, rw.z, rw.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float z = round_bf16(acc[i][e] * rsr[i][e]);  // the bf16 logit
                    if constexpr (TDIV) z = z / temp;
                    if constexpr (LOGP) {  // the processed score z + mask over the row's 16 tile columns
                        const float zp = z + mask_add;
                        const float mx = row16_max(zp);
                        const float sx = row16_sum(fast_exp(fmaxf(zp - mx, -1.0e4f)));
                        const bool own = rl == 4 * i + e;
                        own_m = own ? mx : own_m;
                        own_s = own ? sx : own_s;
                    }
                    float key = smp.p.greedy ? z : z + gumbel_from_bits(wd[e]);
                    key += mask_add;
                    // branch-free: a lane's columns grow with t, so the index tie-break only
                    // ever fires against the initial (-inf, INT_MAX) entry
                    const bool better = (key > bk[i][e]) | ((key == bk[i][e]) & (col < bi[i][e]));
                    bk[i][e] = better ? key : bk[i][e];
                    bi[i][e] = better ? col : bi[i][e];
                }
            }
            if constexpr (LOGP) {  // fold the tile into the owned row's running state
                if (own_m != kNegInf) {
                    const float nm = fmaxf(lm_run, own_m);
                    ls_run = (lm_run == kNegInf ? 0.f : ls_run * fast_exp(lm_run - nm)) + own_s * fast_exp(own_m - nm);
                    lm_run = nm;
                }
            }
        } else if constexpr (EPI == EPI_SILU && !SWH_SILU_ST16) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = round_bf16(acc[i][e] * rsr[i][e]);
                    const float u = __shfl_xor(v, 8, kWave);
                    const int row = m0 + i * 16 + 4 * g + e;
                    if (rl < 8 && row < M) {
                        const int col = t * 8 + rl;
                        const int64_t at = smp.yf ? ((((int64_t)(row >> 4) * (N >> 5) + (col >> 5)) * 64 +
                                                      ((col >> 3) & 3) * 16 + (row & 15)) * 8 + (col & 7))
                                                  : (int64_t)row * ldy + col;
                        y[at] = f32_to_bf16_bits(round_bf16(v / (1.f + expf(-v))) * u);
                    }
                }
        } else if constexpr (EPI == EPI_SILU) {
            // lanes rl < 8 hold gate column t*8+rl, lanes rl+8 the matching up column.
            // Both lanes of a pair can form y = bf16(silu(gate)) * up of their column:
            // the gate lanes take rows 0-31 of the tile, the up lanes rows 32-63, into
            // the wave's 1 KB LDS tile [64 rows][8 columns]; then lane r stores row r's
            // 8 columns (16 contiguous bytes in the fragment order and row-major alike)
            // as one 16-B store instead of 16 scattered 2-B stores.
            uint16_t *yt = reinterpret_cast<uint16_t *>(lds + L.total) + wid * 512;
            const bool gl = rl < 8;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = round_bf16(acc[i][e] * rsr[i][e]);
                    const float u = __shfl_xor(v, 8, kWave);
                    if (gl == (i < 2)) {
                        const float gt = gl ? v : u, up = gl ? u : v;
                        yt[(i * 16 + 4 * g + e) * 8 + (rl & 7)] = f32_to_bf16_bits(round_bf16(gt / (1.f + expf(-gt))) * up);
                    }
                }
            const uint4 yr = *reinterpret_cast<const uint4 *>(yt + lane * 8);
            const int row = m0 + lane, col = t * 8;  // yf: ((row/16 * N/32 + col/32) 64 + row%16 + 16 (col/8 % 4)) 8
            if (row < M) {
                const int64_t at = smp.yf ? (((int64_t)(row >> 4) * (N >> 5) + (col >> 5)) * 64 +
                                             ((col >> 3) & 3) * 16 + (row & 15)) * 8
                                          : (int64_t)row * ldy + col;
                *reinterpret_cast<uint4 *>(y + at) = yr;
            }
        } else {
            // C layout: lane holds rows 16 i + 4 g + e of column rl.  Through the wave's
            // 2 KB LDS tile [64 rows][16 columns], lane r stores row r's 16 columns as
            // two 16-B pieces (not 16 scattered 2-B stores).
            const float bz = BIAS ? bf16_bits_to_f32(bias[t * 16 + rl]) : 0.f;
            uint16_t *yt = reinterpret_cast<uint16_t *>(lds + L.total) + wid * 1024;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    yt[(i * 16 + 4 * g + e) * 16 + rl] = f32_to_bf16_bits(acc[i][e] * rsr[i][e] + bz);
            const uint4 y0 = *reinterpret_cast<const uint4 *>(yt + lane * 16);
            const uint4 y1 = *reinterpret_cast<const uint4 *>(yt + lane * 16 + 8);
            if (m0 + lane < M) {
                uint4 *dst = reinterpret_cast<uint4 *>(y + (int64_t)(m0 + lane) * ldy + t * 16);
                dst[0] = y0;
                dst[1] = y1;
            }
        }
    }
    SWH_GEMM_TRACE(5);
    if constexpr (SAMPLE) {
        // best over the 16 column lanes per wave, then over the workgroup's waves
        // through LDS (the X image is free once every wave is past its tiles):
        // one partial per (row, workgroup) for the finalize
        LmPart *wpart = reinterpret_cast<LmPart *>(xs);  // [NW][64]
        float2 *wsoft = reinterpret_cast<float2 *>(xs + NW * 64 * sizeof(LmPart));  // LOGP: [NW][64]
        __syncthreads();
        if constexpr (LOGP) wsoft[wid * 64 + 16 * (rl >> 2) + 4 * g + (rl & 3)] = float2{lm_run, ls_run};
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float k = bk[i][e];
                int32_t c = bi[i][e];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    const float k2 = __shfl_xor(k, o, kWave);
                    const int32_t c2 = __shfl_xor(c, o, kWave);
                    if (k2 > k || (k2 == k && (uint32_t)c2 < (uint32_t)c)) {
                        k = k2;
                        c = c2;
                    }
                }
                if (rl == 0) wpart[wid * 64 + i * 16 + 4 * g + e] = LmPart{k, c};
            }
        __syncthreads();
        if (tid < 64 && m0 + tid < M) {
            LmPart bpart = wpart[tid];
            for (int q = 1; q < NW; ++q) {
                const LmPart o = wpart[q * 64 + tid];
                if (o.key > bpart.key || (o.key == bpart.key && (uint32_t)o.idx < (uint32_t)bpart.idx)) bpart = o;
            }
            smp.part[(int64_t)(m0 + tid) * smp.pstride + wg] = bpart;
            if constexpr (LOGP) {
                SoftState st = soft_init();
                for (int q = 0; q < NW; ++q) st = soft_merge(st, SoftState{wsoft[q * 64 + tid].x, wsoft[q * 64 + tid].y, 0.f});
                smp.lpart[(int64_t)(m0 + tid) * smp.pstride + wg] = float2{st.m, st.s1};
            }
        }
    }
    SWH_GEMM_TRACE(6);
}

// The next step's input, produced by the finalize (swh_lm_head_sample_step):
// the drawn token's embedding row and its RMSNorm partial sums, and the step
// counter advanced by the last row to finish (ticket) — the three small
// launches embed_gather / step_advance / finalize become one.
struct LmNext {
    const uint16_t *embed;  // [V, H] (null: no gather, no advance)
    uint16_t *x;            // [M, H]
    float *ss;              // [M, H / 16] (nullable)
    int32_t *step;          // advanced once every row has read it
    int32_t *ticket;        // zero at allocation, self-resetting
    int H, M;
};

// Merge the per-wave partials of a row; EOS / pad bookkeeping as
// swh_sample_step's finalize (csrc/sampler.hip).
// LOGP (lpart, out_logp non-null): the row's (max, sum) partials are merged too and
// out_logp[b, step] = z - max - log(sum) for the drawn column's processed score z,
// recovered as key + log(-log(u)) of the same Philox draw (the key itself when greedy):
// within an fp32 rounding of the key (~1e-6 at |z| ~ 10) of the score the logits path sees.
__global__ __launch_bounds__(256) void lm_sample_finalize_kernel(const LmPart *__restrict__ part, int P,
                                                                 swh_sample_params p, const int32_t *__restrict__ step_p,
                                                                 int32_t *__restrict__ finished,
                                                                 int64_t *__restrict__ out_tokens, int64_t out_ld,
                                                                 int64_t *__restrict__ cur_tokens, int V, LmNext nx,
                                                                 const float2 *__restrict__ lpart = nullptr,
                                                                 float *__restrict__ out_logp = nullptr,
                                                                 const uint64_t *__restrict__ rng = nullptr) {
    __shared__ float kk[4];
    __shared__ int32_t ii[4];
    __shared__ float sm[4], ssum[4];
    __shared__ int64_t tok_s;
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool logp = lpart && out_logp;
    float k = kNegInf;
    int32_t c = 0x7fffffff;
    SoftState st = soft_init();
    for (int q = tid; q < P; q += 256) {
        const LmPart v = part[b * P + q];
        if (v.key > k || (v.key == k && (uint32_t)v.idx < (uint32_t)c)) {
            k = v.key;
            c = v.idx;
        }
        if (logp) st = soft_merge(st, SoftState{lpart[b * P + q].x, lpart[b * P + q].y, 0.f});
    }
    if (logp) {
        st = wave_soft(st);
        if (lane == 0) {
            sm[wid] = st.m;
            ssum[wid] = st.s1;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float k2 = __shfl_xor(k, o, kWave);
        const int32_t c2 = __shfl_xor(c, o, kWave);
        if (k2 > k || (k2 == k && (uint32_t)c2 < (uint32_t)c)) {
            k = k2;
            c = c2;
        }
    }
    if (lane == 0) {
        kk[wid] = k;
        ii[wid] = c;
    }
    __syncthreads();
    if (tid == 0) {
        for (int q = 1; q < 4; ++q)
            if (kk[q] > k || (kk[q] == k && (uint32_t)ii[q] < (uint32_t)c)) {
                k = kk[q];
                c = ii[q];
            }
        if (c < 0 || c >= V) c = 0;  // fully masked row (cannot happen with min_tokens_to_keep=1)
        const int32_t step = *step_p;
        if (logp) {
            SoftState r = soft_init();
            for (int q = 0; q < 4; ++q) r = soft_merge(r, SoftState{sm[q], ssum[q], 0.f});
            float z = k;
            if (!p.greedy) {
                const uint64_t seed = rng[0], ctr = rng[1] + (uint64_t)step;
                const U4 w4 = philox4x32_10(U4{(uint32_t)c, (uint32_t)(b >> 2), (uint32_t)ctr, (uint32_t)(ctr >> 32)},
                                            (uint32_t)seed, (uint32_t)(seed >> 32));
                const uint32_t q = (uint32_t)(b & 3);
                const uint32_t bits = q == 0 ? w4.x : q == 1 ? w4.y : q == 2 ? w4.z : w4.w;
                z = k - gumbel_from_bits(bits);
            }
            out_logp[b * out_ld + step] = (z - r.m) - fast_log(r.s1);
        }
        int64_t tok = c;
        if (p.pad_token_id >= 0 && finished[b] != 0) tok = p.pad_token_id;
        bool is_eos = false;
        for (int e = 0; e < p.n_eos && e < 4; ++e) is_eos |= (tok == p.eos_ids[e]);
        if (is_eos) finished[b] = 1;
        out_tokens[b * out_ld + step] = tok;
        if (cur_tokens) cur_tokens[b] = tok;
        tok_s = tok;
    }
    if (!nx.embed) return;
    __syncthreads();
    // the next step's input row: embedding of the drawn token + its RMSNorm partials
    const int64_t id = tok_s;
    const int nch = nx.H / 16;
    for (int ch = tid; ch < nch; ch += 256) {
        const uint4 *src = reinterpret_cast<const uint4 *>(nx.embed + id * nx.H) + 2 * ch;
        const uint4 lo = src[0], hi = src[1];
        uint4 *dst = reinterpret_cast<uint4 *>(nx.x + b * nx.H) + 2 * ch;
        dst[0] = lo;
        dst[1] = hi;
        if (nx.ss) {
            float a[8], e[8];
            unpack16<SWH_BF16>(lo, a);
            unpack16<SWH_BF16>(hi, e);
            float ss = 0.f;
#pragma unroll
            for (int q = 0; q < 8; ++q) ss = fmaf(a[q], a[q], ss);
#pragma unroll
            for (int q = 0; q < 8; ++q) ss = fmaf(e[q], e[q], ss);
            nx.ss[b * nch + ch] = ss;
        }
    }
    if (tid == 0) {  // every row has read *step before its ticket: the last one advances it
        const int t = __hip_atomic_fetch_add(nx.ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (t == nx.M - 1) {
            __hip_atomic_store(nx.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(nx.step, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---------------------------------------------------------------------------
// Attention decode (GQA) on MFMA, swapped orientation: one workgroup (8 waves)
// per (kv head, sequence).  S^T = K Q^T on v_mfma_f32_16x16x32_bf16 (A = 16
// cached keys straight from HBM, B = the GQ <= 16 query heads, zero-padded),
// so each lane holds ONE head (lane & 15) and four keys: the softmax max / sum
// reduce over registers and two lane groups only, and P^T, packed to bf16
// pairwise, is the B operand of O^T = V^T P^T as it stands (no LDS round
// trip).  V^T comes from the wave's V tile in LDS through ds_read_b64_tr_b16
// (4 keys x 1 dim per lane).  Waves take interleaved 16-key blocks; every K/V
// load of a round is issued before the RoPE prologue.
// ---------------------------------------------------------------------------
typedef short bf16x4s __attribute__((ext_vector_type(4)));
#ifndef SWH_ATTN_T128
#define SWH_ATTN_T128 256
#endif
#ifndef SWH_ATTN_T64
#define SWH_ATTN_T64 512
#endif
// Threads of a decode-attention workgroup (one (kv head, row)).  At D = 128 (Llama-3-8B:
// 512 workgroups, 164 VGPRs) four waves let two workgroups share a CU, so one streams
// while the other runs its prologue / merge: 41.3 -> 37.4 us per layer, decode step
// 4857 -> 4737 us (two waves: 42.7, three: 38.1; profiles/r5_att4w_graph.log,
// r5_att2w_graph.log).  At D = 64 (the 0.5B bench, 128 workgroups) eight.
constexpr int attn_threads(int D) { return D == 128 ? SWH_ATTN_T128 : SWH_ATTN_T64; }

__device__ __forceinline__ bf16x4s lds_read_tr16(const uint16_t *p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) bf16x4s *)(const_cast<uint16_t *>(p)));
}

// Per-launch options of the decode attention.  The attention grid covers only
// Hkv x B workgroups (128 of 256 CUs at the bench shape); with `jobs`, extra grid
// rows read the weights of the projections that follow into the Infinity Cache
// (swh_attn_decode_l3) and exit.
struct AttnPrefetch {
    int rows;              // attention rows (B): grid rows past it warm the cache
    const int32_t *prow;   // [B] row whose cache holds this row's prompt keys / values, or null (own row)
    int ofrag = 0;         // output in the fragment order o_proj's register-streamed A operand reads (B % 16 == 0)
    const L3Job *jobs = nullptr;  // Infinity Cache warm-up ranges (grid rows past `rows` read them), or null
    int njobs = 0;
    uint32_t *sink = nullptr;     // >= warm-up workgroups x 512 words, written never in practice
    int nwg = 0;                  // warm-up workgroups wanted (rounded up to whole grid rows)
};

// element (row b, column c) of a [B, K] activation in the fragment order of
// xstream_gemm_kernel's A operand (the act_frag layout): per 16-row group and
// 32-wide k-step one 1 KB run of 64 lanes x 8 consecutive columns
__device__ __forceinline__ int64_t frag_at(int64_t b, int c, int K) {
    return (((b >> 4) * (K >> 5) + (c >> 5)) * 64 + ((c >> 3) & 3) * 16 + (b & 15)) * 8 + (c & 7);
}

// Occupancy at D = 128 (Llama-3-8B), measured (profiles/r5_att_ab.log): 164 VGPRs.  With
// eight waves one workgroup per CU; two per CU by a 128-VGPR bound spill (62 us against
// 41.5 us per launch, Q fragments re-read from LDS 60 us); 4 key blocks per wave per
// round (256 VGPRs) 44.8 us.  Four-wave workgroups (attn_threads) put two on a CU
// without either: 37.4 us.
template <int D, int GQ>
__global__ __launch_bounds__(attn_threads(D)) void attn_decode_kernel(
    const uint16_t *__restrict__ qkv, uint16_t *__restrict__ kc, uint16_t *__restrict__ vc,
    const float *__restrict__ rcos, const float *__restrict__ rsin, const int32_t *__restrict__ plen,
    const int32_t *__restrict__ state, int Hq, int Hkv, int Tmax, float scale, uint16_t *__restrict__ out,
    AttnPrefetch pf) {
    static_assert(GQ <= 16, "a kv head serves at most 16 query heads");
    constexpr int kAttnThreads = attn_threads(D), kAttnWaves = kAttnThreads / 64;
    constexpr int DC = D / 32;                 // 32-dim chunks: k-steps of K Q^T
    constexpr int DB = D / 16;                 // 16-dim blocks of O^T
    constexpr int JB = (D == 64) ? 4 : 2;      // key blocks per wave per round (pairs for P V)
    constexpr int KPR = JB * 16 * kAttnWaves;  // keys per round
    constexpr int HD = D / 2;
    constexpr int VS = D + (D == 64 ? 8 : 16);  // V tile row stride (elements): conflict-free transposed reads
    __shared__ __attribute__((aligned(16))) uint16_t q_s[16 * D];
    __shared__ __attribute__((aligned(16))) uint16_t kn_s[D];
    __shared__ __attribute__((aligned(16))) uint16_t vn_s[D];
    // a wave's V tile (its key loop) and, after its loop, its (acc, m, l) record for the
    // merge share one LDS slot: 2 workgroups per CU fit at D = 128 (78 KB instead of 144)
    constexpr int kRed = 16 * (D + 2) * 4, kVt = 32 * VS * 2;
    constexpr int kSlot = (kRed > kVt ? kRed : kVt) / 16 * 16;
    __shared__ __attribute__((aligned(16))) unsigned char slot_s[kAttnWaves][kSlot];
    auto red_s = [&](int w2, int h) -> float * { return reinterpret_cast<float *>(slot_s[w2]) + h * (D + 2); };

    const int kvh = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;
    SWH_GEMM_TRACE(0);  // phase stamps for tools/attn_probe.py (instrumented build only)
    if ((int)blockIdx.y >= pf.rows) {  // an Infinity Cache warm-up workgroup
        if (pf.jobs)
            l3_warm_share<kAttnThreads>(pf.jobs, pf.njobs, (blockIdx.y - pf.rows) * gridDim.x + blockIdx.x,
                                        (gridDim.y - pf.rows) * gridDim.x, pf.sink);
        return;
    }
    // state[0] = index of the token sampled this step; the input token is state[0] - 1
    const int step = state[0] - 1, P = state[1];
    const int pl = plen[b];
    const int slot_new = P + step;
    const int start = P - pl;
    const int pos = pl + step;
    uint16_t *ob = out + b * (int64_t)Hq * D + kvh * GQ * D;
    if (step < 0 || slot_new >= Tmax || pl < 0 || pl > P) {  // never write outside the cache
        for (int idx = tid; idx < GQ * D; idx += kAttnThreads)  // NaN: fail loudly
            out[pf.ofrag ? frag_at(b, kvh * GQ * D + idx, Hq * D) : b * (int64_t)Hq * D + kvh * GQ * D + idx] = 0x7fc0;
        return;
    }
    const int n = slot_new - start + 1;  // keys incl. the new one (index n-1)
    const int64_t cbase = (b * Hkv + kvh) * (int64_t)Tmax * D;
    const uint16_t *kb = kc + cbase + (int64_t)start * D + g * 8;
    const uint16_t *vb = vc + cbase + (int64_t)start * D + g * 8;
    // prompt keys (index < pl, slots start .. P-1) from the row that holds the group's prompt:
    // the G rows of a GRPO group read one copy (HBM once, the rest from the caches)
    const int64_t prow = pf.prow ? (int64_t)min(max(pf.prow[b], 0), pf.rows - 1) : b;
    const int64_t pbase = (prow * Hkv + kvh) * (int64_t)Tmax * D;
    const uint16_t *kbp = kc + pbase + (int64_t)start * D + g * 8;
    const uint16_t *vbp = vc + pbase + (int64_t)start * D + g * 8;

    // lane (g, c16) loads key c16 of each block, dims 32 c + 8 g: the A fragment of K Q^T
    u32x4 kr[JB][DC], vr[JB][DC];  // vector types: uint4 structs defeat SROA under selects
#define SWH_ATTN_ISSUE(base_)                                                                  \
    _Pragma("unroll") for (int i = 0; i < JB; ++i) {                                           \
        const int k0_ = (base_) + (wid + i * kAttnWaves) * 16;                                 \
        if (k0_ < n) {                                                                         \
            const int kk = max(min(k0_ + c16, n - 2), 0);                                      \
            const uint16_t *ks_ = kk < pl ? kbp : kb, *vs_ = kk < pl ? vbp : vb;               \
            _Pragma("unroll") for (int c = 0; c < DC; ++c) {                                   \
                kr[i][c] = *reinterpret_cast<const u32x4 *>(ks_ + (int64_t)kk * D + c * 32);   \
                vr[i][c] = *reinterpret_cast<const u32x4 *>(vs_ + (int64_t)kk * D + c * 32);   \
            }                                                                                  \
        }                                                                                      \
    }
    SWH_ATTN_ISSUE(0)  // the KV stream is in flight during RoPE
    SWH_GEMM_TRACE(1);

    const uint16_t *row = qkv + b * (int64_t)(Hq + 2 * Hkv) * D;
    for (int idx = tid; idx < (GQ + 1) * HD; idx += kAttnThreads) {
        const int hh = idx / HD, i = idx - hh * HD;
        const float c = rcos[(int64_t)pos * HD + i], s = rsin[(int64_t)pos * HD + i];
        const uint16_t *src = (hh < GQ) ? row + (kvh * GQ + hh) * D : row + (Hq + kvh) * D;
        const float x1 = bf16_bits_to_f32(src[i]), x2 = bf16_bits_to_f32(src[i + HD]);
        const uint16_t o1 = f32_to_bf16_bits(round_bf16(x1 * c) + round_bf16(-x2 * s));
        const uint16_t o2 = f32_to_bf16_bits(round_bf16(x2 * c) + round_bf16(x1 * s));
        if (hh < GQ) {
            q_s[hh * D + i] = o1;
            q_s[hh * D + i + HD] = o2;
        } else {
            kn_s[i] = o1;
            kn_s[i + HD] = o2;
        }
    }
    for (int idx = GQ * D + tid; idx < 16 * D; idx += kAttnThreads) q_s[idx] = 0;
    for (int d = tid; d < D; d += kAttnThreads) vn_s[d] = row[(Hq + Hkv + kvh) * D + d];
    lds_barrier();
    SWH_GEMM_TRACE(2);
    for (int d = tid; d < D; d += kAttnThreads) {  // KV append (nobody reads the slot from memory this step)
        kc[cbase + (int64_t)slot_new * D + d] = kn_s[d];
        vc[cbase + (int64_t)slot_new * D + d] = vn_s[d];
    }

    // B operand of K Q^T: lane holds head c16, dims 32 c + 8 g
    u32x4 qb[DC];
#pragma unroll
    for (int c = 0; c < DC; ++c) qb[c] = *reinterpret_cast<const u32x4 *>(q_s + c16 * D + c * 32 + g * 8);
    float m = kNegInf, l = 0.f;  // of head c16
    f32x4 o[DB];                 // O^T: dims 16 db + 4 g + r, head c16
#pragma unroll
    for (int d = 0; d < DB; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint16_t *vt = reinterpret_cast<uint16_t *>(slot_s[wid]);

    for (int base = 0; base < n; base += KPR) {
        if (base) {
            SWH_ATTN_ISSUE(base)
        }
        f32x4 sc[JB];  // S^T: keys k0 + 4 g + r, head c16
        float mx = m;
#pragma unroll
        for (int i = 0; i < JB; ++i) {
            const int k0 = base + (wid + i * kAttnWaves) * 16;
            sc[i] = f32x4{kNegInf, kNegInf, kNegInf, kNegInf};
            if (k0 < n) {  // wave-uniform
                const bool fresh = (k0 + c16 == n - 1);  // the new key/value: from LDS, not the cache
#pragma unroll
                for (int c = 0; c < DC; ++c) {
                    const u32x4 kn = *reinterpret_cast<const u32x4 *>(kn_s + c * 32 + g * 8);
                    const u32x4 vn = *reinterpret_cast<const u32x4 *>(vn_s + c * 32 + g * 8);
                    kr[i][c] = fresh ? kn : kr[i][c];
                    vr[i][c] = fresh ? vn : vr[i][c];
                }
                f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int c = 0; c < DC; ++c)
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kr[i][c]),
                                                                  __builtin_bit_cast(bf16x8, qb[c]), acc, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    sc[i][r] = (k0 + 4 * g + r < n) ? acc[r] * scale : kNegInf;
                    mx = fmaxf(mx, sc[i][r]);
                }
            }
        }
        // online softmax of head c16: its keys sit in 4 registers x JB blocks x the 4 lane groups
        mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
        mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
        const float corr = (mx == kNegInf) ? 1.f : expf(m - mx);
        l *= corr;
#pragma unroll
        for (int d = 0; d < DB; ++d) o[d] *= corr;
        m = mx;
        // P V: blocks in pairs -> 32 keys per MFMA; P^T (bf16 pairs) is the B operand as it stands
#pragma unroll
        for (int i = 0; i < JB; i += 2) {
            const int k0 = base + (wid + i * kAttnWaves) * 16;
            const int k1 = base + (wid + (i + 1) * kAttnWaves) * 16;
            if (k0 < n) {  // wave-uniform
                float pj[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    pj[r] = (mx == kNegInf) ? 0.f : expf(sc[i][r] - mx);
                    pj[4 + r] = (mx == kNegInf) ? 0.f : expf(sc[i + 1][r] - mx);
                    l += pj[r] + pj[4 + r];
                }
                // the pair's V rows into the wave's tile (rows 0-15: block i, 16-31: block i+1; zeros past n)
#pragma unroll
                for (int c = 0; c < DC; ++c) {
                    *reinterpret_cast<u32x4 *>(vt + c16 * VS + c * 32 + g * 8) = vr[i][c];
                    *reinterpret_cast<u32x4 *>(vt + (16 + c16) * VS + c * 32 + g * 8) =
                        (k1 < n) ? vr[i + 1][c] : u32x4{0u, 0u, 0u, 0u};
                }
                uint32_t pb[4];
#pragma unroll
                for (int h = 0; h < 4; ++h)
                    pb[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{pj[2 * h], pj[2 * h + 1]}, bf16x2));
                const bf16x8 pbf = __builtin_bit_cast(bf16x8, u32x4{pb[0], pb[1], pb[2], pb[3]});
                // V^T fragment: lane (g, c16) <- dims 16 db + c16 of keys {4 g .. 4 g + 3} and {16 + 4 g ..}
                const int q = c16 >> 2, pq = c16 & 3;
#pragma unroll
                for (int d = 0; d < DB; ++d) {
                    const bf16x4s lo = lds_read_tr16(vt + (4 * g + q) * VS + d * 16 + 4 * pq);
                    const bf16x4s hi = lds_read_tr16(vt + (16 + 4 * g + q) * VS + d * 16 + 4 * pq);
                    const bf16x8 va = __builtin_bit_cast(
                        bf16x8, u32x4{__builtin_bit_cast(uint2, lo).x, __builtin_bit_cast(uint2, lo).y,
                                      __builtin_bit_cast(uint2, hi).x, __builtin_bit_cast(uint2, hi).y});
                    o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pbf, o[d], 0, 0, 0);
                }
            }
        }
    }
    SWH_GEMM_TRACE(3);
    // row sums across the 4 lane groups, then the waves merge through LDS (the record
    // overwrites this wave's own V tile: its last transposed reads must retire first)
    l += __shfl_xor(l, 16, kWave);
    l += __shfl_xor(l, 32, kWave);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    float *rec = red_s(wid, c16);
#pragma unroll
    for (int d = 0; d < DB; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) rec[d * 16 + 4 * g + r] = o[d][r];
    if (g == 0) {
        rec[D] = m;
        rec[D + 1] = l;
    }
    __syncthreads();
    SWH_GEMM_TRACE(4);
    auto merged = [&](int h, int d) -> uint16_t {  // the waves' (m, l, acc) of head h, dim d
        float mxw = kNegInf;
#pragma unroll
        for (int w2 = 0; w2 < kAttnWaves; ++w2) mxw = fmaxf(mxw, red_s(w2, h)[D]);
        float Ls = 0.f, A = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < kAttnWaves; ++w2) {
            const float *rw = red_s(w2, h);
            const float mq = rw[D];
            if (mq == kNegInf) continue;
            const float cq = expf(mq - mxw);
            Ls = fmaf(rw[D + 1], cq, Ls);
            A = fmaf(rw[d], cq, A);
        }
        return f32_to_bf16_bits(A / Ls);
    };
    if (pf.ofrag) {
        // one element per thread as below; lanes 8j .. 8j+7 hold 8 consecutive dims
        // (GQ * D % 64 == 0: whole waves per pass), gathered by shuffles into lane 8j,
        // which stores them as one 16-B piece at their fragment-order place
        for (int idx = tid; idx < GQ * D; idx += kAttnThreads) {
            const int h = idx / D, d = idx - h * D;
            const uint32_t v = merged(h, d);
            const uint32_t p2 = v | (__shfl_down(v, 1, kWave) << 16);
            const uint32_t p4 = __shfl_down(p2, 2, kWave);
            const uint32_t p6 = __shfl_down(p2, 4, kWave), p8 = __shfl_down(p2, 6, kWave);
            if ((lane & 7) == 0)
                *reinterpret_cast<uint4 *>(out + frag_at(b, (kvh * GQ + h) * D + d, Hq * D)) = uint4{p2, p4, p6, p8};
        }
    } else {
        for (int idx = tid; idx < GQ * D; idx += kAttnThreads) {
            const int h = idx / D, d = idx - h * D;
            ob[idx] = merged(h, d);
        }
    }
    SWH_GEMM_TRACE(5);
#undef SWH_ATTN_ISSUE
}

// ---------------------------------------------------------------------------
// Row-pair decode attention (D = 128, 2 GQ <= 16: Llama-3-8B): one 8-wave workgroup
// per (kv head, two consecutive rows).  The MFMA's 16 query columns hold both rows'
// heads (row A in columns 0 .. GQ-1, row B in GQ .. 2 GQ-1), so when the rows share a
// GRPO group's prompt (prompt_row and prompt length equal) its keys and values are
// loaded ONCE and scored for both rows; each row's own keys follow with the other
// row's columns masked to -inf (their online-softmax state untouched).  One wave of
// 256 workgroups instead of two of 512 halves the exposed argument / RoPE / merge
// phases as well (timing probe: 37.8 -> 32.3 us per layer, profiles/r5_pair_graph.log).
// Same per-column arithmetic as attn_decode_kernel (scores, online softmax, P V,
// fixed-order wave merge), with the keys visited in another order.
// ---------------------------------------------------------------------------
template <int D, int GQ>
__global__ __launch_bounds__(512) void attn_decode_pair_kernel(
    const uint16_t *__restrict__ qkv, uint16_t *__restrict__ kc, uint16_t *__restrict__ vc,
    const float *__restrict__ rcos, const float *__restrict__ rsin, const int32_t *__restrict__ plen,
    const int32_t *__restrict__ state, int Hq, int Hkv, int Tmax, float scale, uint16_t *__restrict__ out,
    AttnPrefetch pf) {
    static_assert(2 * GQ <= 16, "two rows' query heads in the 16 MFMA columns");
    constexpr int NT = 512, NW = NT / 64;
    constexpr int DC = D / 32, DB = D / 16, JB = 2, KPR = JB * 16 * NW, HD = D / 2;
    constexpr int VS = D + (D == 64 ? 8 : 16);
    __shared__ __attribute__((aligned(16))) uint16_t q_s[16 * D];
    __shared__ __attribute__((aligned(16))) uint16_t kn_s[2][D];
    __shared__ __attribute__((aligned(16))) uint16_t vn_s[2][D];
    constexpr int kRed = 16 * (D + 2) * 4, kVt = 32 * VS * 2;
    constexpr int kSlot = (kRed > kVt ? kRed : kVt) / 16 * 16;
    __shared__ __attribute__((aligned(16))) unsigned char slot_s[NW][kSlot];
    auto red_s = [&](int w2, int h) -> float * { return reinterpret_cast<float *>(slot_s[w2]) + h * (D + 2); };

    const int kvh = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;
    const int npairs = (pf.rows + 1) / 2;
    if ((int)blockIdx.y >= npairs) {  // an Infinity Cache warm-up workgroup
        if (pf.jobs)
            l3_warm_share<NT>(pf.jobs, pf.njobs, (blockIdx.y - npairs) * gridDim.x + blockIdx.x,
                              (gridDim.y - npairs) * gridDim.x, pf.sink);
        return;
    }
    const int step = state[0] - 1, P = state[1];
    const int slot_new = P + step;
    // never write outside the cache: a row with an out-of-range length or step gets NaN
    // (fails loudly) and no KV append; its partner row still runs, alone
    const int64_t b0 = 2 * (int64_t)blockIdx.y;
    const bool has1 = b0 + 1 < pf.rows;
    const int pl0 = plen[b0], pl1 = has1 ? plen[b0 + 1] : 0;
    const bool ok0 = !(step < 0 || slot_new >= Tmax || pl0 < 0 || pl0 > P);
    const bool ok1 = has1 && !(step < 0 || slot_new >= Tmax || pl1 < 0 || pl1 > P);
    for (int r = 0; r < (has1 ? 2 : 1); ++r) {
        if (r ? ok1 : ok0) continue;
        const int64_t b = b0 + r;
        for (int idx = tid; idx < GQ * D; idx += NT)
            out[pf.ofrag ? frag_at(b, kvh * GQ * D + idx, Hq * D) : b * (int64_t)Hq * D + kvh * GQ * D + idx] = 0x7fc0;
    }
    if (!ok0 && !ok1) return;
    const int64_t bA = ok0 ? b0 : b0 + 1;
    const bool hasB = ok0 && ok1;
    const int64_t bB = hasB ? bA + 1 : bA;
    const int plA = ok0 ? pl0 : pl1, plB = hasB ? pl1 : plA;
    const int64_t prA = pf.prow ? (int64_t)min(max(pf.prow[bA], 0), pf.rows - 1) : bA;
    const int64_t prB = pf.prow ? (int64_t)min(max(pf.prow[bB], 0), pf.rows - 1) : bB;
    const bool shared = hasB && prA == prB && plA == plB && plA > 0;  // one prompt for both rows
    const int nA = slot_new - (P - plA) + 1, nB = slot_new - (P - plB) + 1;  // keys incl. the new one
    auto cbase = [&](int64_t r) -> int64_t { return (r * Hkv + kvh) * (int64_t)Tmax * D; };
    const int64_t cbA = cbase(bA), cbB = cbase(bB);

    // key segments: [lo, hi) of a row's key numbering (prompt keys first), read from the
    // prompt row's cache below pl and the row's own cache from pl on; columns [clo, chi)
    struct Seg {
        int lo, hi, pl, n, clo, chi, fresh;  // fresh: 0 none, 1 row A's new key, 2 row B's
        const uint16_t *kb, *vb, *kbp, *vbp;
    };
    const int stA = P - plA, stB = P - plB;
    const uint16_t *kA = kc + cbA + (int64_t)stA * D + g * 8, *vA = vc + cbA + (int64_t)stA * D + g * 8;
    const uint16_t *kB = kc + cbB + (int64_t)stB * D + g * 8, *vB = vc + cbB + (int64_t)stB * D + g * 8;
    const uint16_t *kpA = kc + cbase(prA) + (int64_t)stA * D + g * 8, *vpA = vc + cbase(prA) + (int64_t)stA * D + g * 8;
    const uint16_t *kpB = kc + cbase(prB) + (int64_t)stB * D + g * 8, *vpB = vc + cbase(prB) + (int64_t)stB * D + g * 8;
    // A row's keys are always visited as its prompt [0, pl), then its own [pl, n), with the
    // same round boundaries, so a column's result does not depend on whether the pair
    // shares its prompt (shared: one prompt segment scored for both rows' columns).  No
    // dynamic indexing (a segment array lived in scratch): the segments as values.
    const Seg sP{0, plA, plA, 0x7fffffff, 0, 2 * GQ, 0, kA, vA, kpA, vpA};
    const Seg sAp{0, plA, plA, 0x7fffffff, 0, GQ, 0, kA, vA, kpA, vpA};
    const Seg sAo{plA, nA, plA, nA, 0, GQ, 1, kA, vA, kpA, vpA};
    const Seg sBp{0, hasB ? plB : 0, plB, 0x7fffffff, GQ, 2 * GQ, 0, kB, vB, kpB, vpB};
    const Seg sBo{plB, hasB ? nB : plB, plB, nB, GQ, 2 * GQ, 2, kB, vB, kpB, vpB};
    const Seg s0 = shared ? sP : sAp;

    u32x4 kr[JB][DC], vr[JB][DC];
    // A run visits the 16-key blocks of a virtual list: part X's keys [X.lo, X.hi) padded to
    // whole blocks, then part Y's [Y.lo, Y.hi); each block belongs to one part (wave-uniform),
    // so both rows' own keys share rounds.  blk(k0v) -> the part's Seg and key index.
#define SWH_PAIR_BLOCK(X_, Y_, k0v_, S_, k0_)                                                     \
    const int p1_ = ((X_).hi - (X_).lo + 15) / 16 * 16;                                           \
    const bool iny_ = (k0v_) >= p1_;                                                              \
    const Seg S_ = iny_ ? (Y_) : (X_);                                                            \
    const int k0_ = iny_ ? (Y_).lo + (k0v_) - p1_ : (X_).lo + (k0v_);
#define SWH_PAIR_ISSUE(X_, Y_, base_)                                                             \
    _Pragma("unroll") for (int i = 0; i < JB; ++i) {                                              \
        SWH_PAIR_BLOCK(X_, Y_, (base_) + (wid + i * NW) * 16, S_, k0_)                            \
        if (k0_ < S_.hi) {                                                                        \
            const int kk = max(min(k0_ + c16, min(S_.hi, S_.n - 1) - 1), 0);                      \
            const uint16_t *ks_ = kk < S_.pl ? S_.kbp : S_.kb;                                    \
            const uint16_t *vs_ = kk < S_.pl ? S_.vbp : S_.vb;                                    \
            _Pragma("unroll") for (int c = 0; c < DC; ++c) {                                      \
                kr[i][c] = *reinterpret_cast<const u32x4 *>(ks_ + (int64_t)kk * D + c * 32);      \
                vr[i][c] = *reinterpret_cast<const u32x4 *>(vs_ + (int64_t)kk * D + c * 32);      \
            }                                                                                     \
        }                                                                                         \
    }
    const Seg s_none{0, 0, 0, 0, 0, 0, 0, kA, vA, kA, vA};
    SWH_PAIR_ISSUE(s0, s_none, 0)  // the first segment's KV stream is in flight during RoPE

    // RoPE of both rows' query heads (columns 0 .. 2 GQ - 1) and new keys; new values
    for (int idx = tid; idx < 2 * (GQ + 1) * HD; idx += NT) {
        const int r = idx / ((GQ + 1) * HD), rem = idx - r * (GQ + 1) * HD;
        const int hh = rem / HD, i = rem - hh * HD;
        const int64_t b = r ? bB : bA;
        const int pos = (r ? plB : plA) + step;
        const uint16_t *row = qkv + b * (int64_t)(Hq + 2 * Hkv) * D;
        const float c = rcos[(int64_t)pos * HD + i], s = rsin[(int64_t)pos * HD + i];
        const uint16_t *src = (hh < GQ) ? row + (kvh * GQ + hh) * D : row + (Hq + kvh) * D;
        const float x1 = bf16_bits_to_f32(src[i]), x2 = bf16_bits_to_f32(src[i + HD]);
        const uint16_t o1 = f32_to_bf16_bits(round_bf16(x1 * c) + round_bf16(-x2 * s));
        const uint16_t o2 = f32_to_bf16_bits(round_bf16(x2 * c) + round_bf16(x1 * s));
        if (hh < GQ) {
            q_s[(r * GQ + hh) * D + i] = o1;
            q_s[(r * GQ + hh) * D + i + HD] = o2;
        } else {
            kn_s[r][i] = o1;
            kn_s[r][i + HD] = o2;
        }
    }
    for (int idx = 2 * GQ * D + tid; idx < 16 * D; idx += NT) q_s[idx] = 0;
    for (int d = tid; d < 2 * D; d += NT) {
        const int r = d / D;
        vn_s[r][d - r * D] = qkv[(r ? bB : bA) * (int64_t)(Hq + 2 * Hkv) * D + (Hq + Hkv + kvh) * D + d - r * D];
    }
    lds_barrier();
    for (int d = tid; d < (hasB ? 2 : 1) * D; d += NT) {  // KV append of both rows
        const int r = d / D, e = d - r * D;
        const int64_t cb = r ? cbB : cbA;
        kc[cb + (int64_t)slot_new * D + e] = kn_s[r][e];
        vc[cb + (int64_t)slot_new * D + e] = vn_s[r][e];
    }

    u32x4 qb[DC];
#pragma unroll
    for (int c = 0; c < DC; ++c) qb[c] = *reinterpret_cast<const u32x4 *>(q_s + c16 * D + c * 32 + g * 8);
    float m = kNegInf, l = 0.f;
    f32x4 o[DB];
#pragma unroll
    for (int d = 0; d < DB; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint16_t *vt = reinterpret_cast<uint16_t *>(slot_s[wid]);

    bool first = true;
    auto run = [&](const Seg &X, const Seg &Y) __attribute__((always_inline)) {
        const int vlen = (X.hi - X.lo + 15) / 16 * 16 + (Y.hi - Y.lo);
        if (X.hi <= X.lo && Y.hi <= Y.lo) return;
        for (int base = 0; base < vlen; base += KPR) {
            if (!first) {
                SWH_PAIR_ISSUE(X, Y, base)
            }
            first = false;
            f32x4 sc[JB];
            float mx = m;
            bool live[JB];  // block i holds some key (wave-uniform)
#pragma unroll
            for (int i = 0; i < JB; ++i) {
                SWH_PAIR_BLOCK(X, Y, base + (wid + i * NW) * 16, S, k0)
                const bool colv = c16 >= S.clo && c16 < S.chi;  // this lane's column scores these keys
                sc[i] = f32x4{kNegInf, kNegInf, kNegInf, kNegInf};
                live[i] = k0 < S.hi;
                if (k0 < S.hi) {  // wave-uniform
                    const bool fresh = S.fresh && (k0 + c16 == S.n - 1);  // the new key/value, from LDS
                    const int fr = S.fresh == 2 ? 1 : 0;
#pragma unroll
                    for (int c = 0; c < DC; ++c) {
                        const u32x4 kn = *reinterpret_cast<const u32x4 *>(kn_s[fr] + c * 32 + g * 8);
                        const u32x4 vn = *reinterpret_cast<const u32x4 *>(vn_s[fr] + c * 32 + g * 8);
                        kr[i][c] = fresh ? kn : kr[i][c];
                        vr[i][c] = fresh ? vn : vr[i][c];
                    }
                    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int c = 0; c < DC; ++c)
                        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kr[i][c]),
                                                                      __builtin_bit_cast(bf16x8, qb[c]), acc, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        sc[i][r] = (colv && k0 + 4 * g + r < S.hi) ? acc[r] * scale : kNegInf;
                        mx = fmaxf(mx, sc[i][r]);
                    }
                }
            }
            mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
            mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
            const float corr = (mx == kNegInf) ? 1.f : expf(m - mx);
            l *= corr;
#pragma unroll
            for (int d = 0; d < DB; ++d) o[d] *= corr;
            m = mx;
#pragma unroll
            for (int i = 0; i < JB; i += 2) {
                if (live[i] || live[i + 1]) {  // wave-uniform
                    float pj[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        pj[r] = (mx == kNegInf) ? 0.f : expf(sc[i][r] - mx);
                        pj[4 + r] = (mx == kNegInf) ? 0.f : expf(sc[i + 1][r] - mx);
                        l += pj[r] + pj[4 + r];
                    }
#pragma unroll
                    for (int c = 0; c < DC; ++c) {
                        *reinterpret_cast<u32x4 *>(vt + c16 * VS + c * 32 + g * 8) =
                            live[i] ? vr[i][c] : u32x4{0u, 0u, 0u, 0u};
                        *reinterpret_cast<u32x4 *>(vt + (16 + c16) * VS + c * 32 + g * 8) =
                            live[i + 1] ? vr[i + 1][c] : u32x4{0u, 0u, 0u, 0u};
                    }
                    uint32_t pb[4];
#pragma unroll
                    for (int h = 0; h < 4; ++h)
                        pb[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{pj[2 * h], pj[2 * h + 1]}, bf16x2));
                    const bf16x8 pbf = __builtin_bit_cast(bf16x8, u32x4{pb[0], pb[1], pb[2], pb[3]});
                    const int q = c16 >> 2, pq = c16 & 3;
#pragma unroll
                    for (int d = 0; d < DB; ++d) {
                        const bf16x4s lo = lds_read_tr16(vt + (4 * g + q) * VS + d * 16 + 4 * pq);
                        const bf16x4s hi = lds_read_tr16(vt + (16 + 4 * g + q) * VS + d * 16 + 4 * pq);
                        const bf16x8 va = __builtin_bit_cast(
                            bf16x8, u32x4{__builtin_bit_cast(uint2, lo).x, __builtin_bit_cast(uint2, lo).y,
                                          __builtin_bit_cast(uint2, hi).x, __builtin_bit_cast(uint2, hi).y});
                        o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pbf, o[d], 0, 0, 0);
                    }
                }
            }
        }
    };
    run(s0, s_none);
    first = false;  // s0 may be empty (a zero-length prompt): the next run issues its own first round
    if (!shared) run(sBp, s_none);
    run(sAo, sBo);  // both rows' own keys: A's blocks, then B's, sharing rounds
#undef SWH_PAIR_ISSUE
#undef SWH_PAIR_BLOCK
    l += __shfl_xor(l, 16, kWave);
    l += __shfl_xor(l, 32, kWave);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    float *rec = red_s(wid, c16);
#pragma unroll
    for (int d = 0; d < DB; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) rec[d * 16 + 4 * g + r] = o[d][r];
    if (g == 0) {
        rec[D] = m;
        rec[D + 1] = l;
    }
    __syncthreads();
    auto merged = [&](int h, int d) -> uint16_t {  // the waves' (m, l, acc) of column h, dim d
        float mxw = kNegInf;
#pragma unroll
        for (int w2 = 0; w2 < NW; ++w2) mxw = fmaxf(mxw, red_s(w2, h)[D]);
        float Ls = 0.f, A = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < NW; ++w2) {
            const float *rw = red_s(w2, h);
            const float mq = rw[D];
            if (mq == kNegInf) continue;
            const float cq = expf(mq - mxw);
            Ls = fmaf(rw[D + 1], cq, Ls);
            A = fmaf(rw[d], cq, A);
        }
        return f32_to_bf16_bits(A / Ls);
    };
    const int nrow = hasB ? 2 : 1;
    if (pf.ofrag) {
        for (int idx = tid; idx < nrow * GQ * D; idx += NT) {  // GQ * D % 64 == 0: whole waves per row
            const int h = idx / D, d = idx - h * D, r = h / GQ;
            const uint32_t v = merged(h, d);
            const uint32_t p2 = v | (__shfl_down(v, 1, kWave) << 16);
            const uint32_t p4 = __shfl_down(p2, 2, kWave);
            const uint32_t p6 = __shfl_down(p2, 4, kWave), p8 = __shfl_down(p2, 6, kWave);
            if ((lane & 7) == 0)
                *reinterpret_cast<uint4 *>(out + frag_at(bA + r, (kvh * GQ + h - r * GQ) * D + d, Hq * D)) =
                    uint4{p2, p4, p6, p8};
        }
    } else {
        for (int idx = tid; idx < nrow * GQ * D; idx += NT) {
            const int h = idx / D, d = idx - h * D, r = h / GQ;
            out[(bA + r) * (int64_t)Hq * D + (kvh * GQ + h - r * GQ) * D + d] = merged(h, d);
        }
    }
}

template <int D, int GQ>
int launch_attn(const uint16_t *q, uint16_t *kc, uint16_t *vc, const float *rc, const float *rs, const int32_t *pl,
                const int32_t *st, int64_t B, int Hq, int Hkv, int Tmax, float scale, uint16_t *o, hipStream_t s,
                const AttnPrefetch &pf) {
    // warm-up rows: whole grid rows of Hkv workgroups
    int64_t extra = 0;
    if (pf.jobs) {
        extra = (pf.nwg + Hkv - 1) / Hkv;
        if (B + extra > 65535) extra = 0;
    }
    if constexpr (D == 128 && 2 * GQ <= 16) {
        if (launch_policy().attn_pair) {  // row pairs: (B + 1) / 2 grid rows, then the warm-up rows
            const int64_t pairs = (B + 1) / 2;
            if (pairs + extra > 65535) extra = 0;
            attn_decode_pair_kernel<D, GQ><<<dim3((unsigned)Hkv, (unsigned)(pairs + extra)), 512, 0, s>>>(
                q, kc, vc, rc, rs, pl, st, Hq, Hkv, Tmax, scale, o, pf);
            return launch_status();
        }
    }
    attn_decode_kernel<D, GQ><<<dim3((unsigned)Hkv, (unsigned)(B + extra)), attn_threads(D), 0, s>>>(
        q, kc, vc, rc, rs, pl, st, Hq, Hkv, Tmax, scale, o, pf);
    return launch_status();
}

template <int D>
int attn_dispatch_gq(int gq, const uint16_t *q, uint16_t *kc, uint16_t *vc, const float *rc, const float *rs,
                     const int32_t *pl, const int32_t *st, int64_t B, int Hq, int Hkv, int Tmax, float scale,
                     uint16_t *o, hipStream_t s, const AttnPrefetch &pf) {
    switch (gq) {
    case 1: return launch_attn<D, 1>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s, pf);
    case 2: return launch_attn<D, 2>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s, pf);
    case 3: return launch_attn<D, 3>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s, pf);
    case 4: return launch_attn<D, 4>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s, pf);
    case 5: return launch_attn<D, 5>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s, pf);
    case 6: return launch_attn<D, 6>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s, pf);
    case 7: return launch_attn<D, 7>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s, pf);
    case 8: return launch_attn<D, 8>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s, pf);
    default: return SWH_E_ARG;
    }
}

// ---- GEMM launch configuration -------------------------------------------
// The smallest K routed to csrc/wide_gemm.hip and whether that path is on come from
// the launch policy (swh_set_launch_policy; the DecodeEngine reads the same policy to
// choose its packed projections), read per call on the host (at graph capture).

struct GemmCfg {
    int ms, cb, nw, s, gx;  // 16-row blocks, 16-col blocks (tile), waves, K split, grid.x
    bool persist;
    int wn = 1;             // column groups: a wave computes cb / wn column blocks over K / (nw / wn)
    int fw = 0;             // weights in the swh_frag_pack layout
    int xf = 0;             // X (the SiLU activation) in the same fragment order (xstream only)
};

// 8 waves in every geometry: more k-steps in flight per CU (down 14.9 -> 11.5 us,
// qkv 7.0 -> 6.3 us against 4 waves for 16- and 32-row tiles; tools/bench_decode.py --ku)
inline int gemm_waves(int) { return 8; }

// Modelled launch time (us) of one geometry — measured shape of the cost on
// MI355X (tools/gemm_probe.py, tools/bench_decode.py --sweep): a fixed
// ~3 us, the bytes one CU pulls through its load path at ~60 GB/s (weights in
// fragment order count twice), ~1 us per 10k elements of in-LDS RMSNorm,
// +9 us for a cross-workgroup split, +3 us per extra wave of workgroups.
double gemm_cost(const GemmCfg &c, int64_t M, int64_t wcols, int64_t K, int nm) {
    const int64_t MR = 16 * c.ms, KS = K / 32, ncu = cu_count();
    const int64_t krmax = (KS + c.s - 1) / c.s * 32;
    const GemmLds L = gemm_lds(c.cb, (int)MR, c.nw, (int)krmax, (int)K, nm, c.persist, c.wn);
    if (L.total > 160 * 1024) return 1e30;
    if (c.cb % c.wn || c.nw % c.wn || MR * c.cb * 2 > 2 * 64 * c.nw) return 1e30;  // epilogue: <= 2 groups / thread
    const int64_t ncb = wcols / (16 * c.cb), nmt = (M + MR - 1) / MR;
    const int64_t xbytes = MR * krmax * 2, wbytes = 2 * 16 * c.cb * krmax * 2;
    if (c.persist) {
        const int64_t wgs = c.gx, per = (ncb + wgs / nmt - 1) / (wgs / nmt);
        return 3.0 + (xbytes + per * wbytes) / 60e3;
    }
    const int64_t wgs = 8 * nmt * ((ncb + 7) / 8) * c.s;
    int64_t res = (160 * 1024) / L.total;
    res = res < 1 ? 1 : (res > 2 ? 2 : res);
    const int64_t per_cu = (wgs + ncu - 1) / ncu, waves = (wgs + ncu * res - 1) / (ncu * res);
    const double norm_us = nm == 1 ? (double)(MR * krmax) / 10e3 : 0.0;  // in-LDS RMSNorm pass
    return 3.0 + per_cu * ((xbytes + wbytes) / 60e3 + norm_us) + (c.s > 1 ? 9.0 : 0.0) + (waves - 1) * 3.0;
}

GemmCfg pick_cfg(int64_t M, int64_t wcols, int64_t K, bool silu, int nm) {
    const int64_t KS = K / 32, align = silu ? 2 : 1, ncu = cu_count();
    GemmCfg best{4, 4, 8, 1, 0, false};
    double best_cost = 1e31;
    for (int ms : {1, 2, 4})
        for (int cb : {1, 2, 4}) {
            if (wcols % (16 * cb * align)) continue;
            for (int sp = 1; sp <= 8; ++sp) {
                if (sp > KS) break;
                GemmCfg c{ms, cb, gemm_waves(ms), sp, 0, false};
                const double t = gemm_cost(c, M, wcols, K, nm);
                if (t < best_cost) {
                    best_cost = t;
                    best = c;
                }
            }
        }
    // persistent: all 64 rows, 32-column blocks, grid = the CUs, weights streamed once
    const int64_t nmt64 = (M + 63) / 64;
    if (wcols % (32 * align) == 0 && ncu / nmt64 >= 1) {
        GemmCfg c{4, 2, 8, 1, (int)((ncu / nmt64) * nmt64), true};
        if (c.gx > wcols / 32 * nmt64) c.gx = (int)(wcols / 32 * nmt64);
        if (gemm_cost(c, M, wcols, K, nm) < best_cost) best = c;
    }
    const swh_launch_policy pol = launch_policy();
    if (pol.gemm_ms) {  // geometry override of the launch policy (tests / A/B)
        const int a = pol.gemm_ms, b = pol.gemm_cb, d = pol.gemm_s, pz = pol.gemm_persist, wn = pol.gemm_wn;
        if ((a == 1 || a == 2 || a == 4) && (b == 1 || b == 2 || b == 4) && d >= 1 && d <= KS && d <= 8 &&
            wcols % (16 * b * align) == 0 && !(pz && d != 1) && (wn == 1 || wn == 2 || wn == 4)) {
            const int64_t nmt = (M + 16 * a - 1) / (16 * a);
            GemmCfg c{a, b, gemm_waves(a), d, 0, pz != 0, wn};
            if (c.persist) {
                const int64_t per = ncu / nmt > 0 ? ncu / nmt : 1, ncb = wcols / (16 * b);
                c.gx = (int)((per < ncb ? per : ncb) * nmt);
            }
            if (gemm_cost(c, M, wcols, K, nm) < 1e29) best = c;
        }
    }
    if (!best.persist) best.gx = (int)(8 * ((M + 16 * best.ms - 1) / (16 * best.ms)) * ((wcols / (16 * best.cb) + 7) / 8));
    // one column block per wave (column groups split the waves, each group splits K):
    // a 4x smaller LDS merge; gate/up 14.7 -> 12.3 us (tools/bench_decode.py --ku)
    if (!pol.gemm_ms && !best.persist && best.cb > 1 && best.nw % best.cb == 0 &&
        gemm_cost(GemmCfg{best.ms, best.cb, best.nw, best.s, best.gx, false, best.cb}, M, wcols, K, nm) < 1e29)
        best.wn = best.cb;
    if (pol.gemm_nw) {  // policy override: waves per workgroup (16: cb == 1 only)
        const int v = pol.gemm_nw;
        if ((v == 4 || v == 8 || (v == 16 && best.cb == best.wn)) &&
            gemm_cost(GemmCfg{best.ms, best.cb, v, best.s, best.gx, best.persist, best.wn}, M, wcols, K, nm) < 1e29)
            best.nw = v;
    }
    return best;
}

int64_t slab_bytes(const GemmCfg &c, int64_t M, int64_t wcols) {
    if (c.s == 1) return 0;
    const int64_t MR = 16 * c.ms, nmt = (M + MR - 1) / MR;
    return nmt * wcols * c.s * MR * (int64_t)sizeof(float);  // tiles * NB == nmt * wcols
}

template <int CB, int MS, int NM, int EPI, bool BIAS, int MAXT, int KL>
int launch_gemm_kl(const GemmCfg &c, dim3 grid, size_t lds, hipStream_t s, const uint16_t *X, const uint16_t *W,
                   int m, int n, int k, const uint16_t *NWt, float eps, const float *ss_in, const uint16_t *Bs,
                   uint16_t *R, float *ss_out, uint16_t *Y, int ld, float *slab, int *ctr) {
    if (!lds_opt_in<&decode_gemm_kernel<CB, MS, NM, EPI, BIAS, MAXT, KL>>()) return SWH_E_LAUNCH;  // > 64 KB LDS
    decode_gemm_kernel<CB, MS, NM, EPI, BIAS, MAXT, KL><<<grid, 64u * c.nw, lds, s>>>(
        X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr, c.persist ? 1 : 0, c.wn, c.fw);
    return launch_status();
}

template <int CB, int MS, int NM, int EPI, bool BIAS, int MAXT>
int launch_gemm(const GemmCfg &c, dim3 grid, size_t lds, hipStream_t s, const uint16_t *X, const uint16_t *W, int m,
                int n, int k, const uint16_t *NWt, float eps, const float *ss_in, const uint16_t *Bs, uint16_t *R,
                float *ss_out, uint16_t *Y, int ld, float *slab, int *ctr) {
    // residual projections: o_proj (K = H) and down_proj (K = I) get distinct names
    if (EPI == EPI_RESIDUAL && k > 1024)
        return launch_gemm_kl<CB, MS, NM, EPI, BIAS, MAXT, 1>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R,
                                                              ss_out, Y, ld, slab, ctr);
    return launch_gemm_kl<CB, MS, NM, EPI, BIAS, MAXT, 0>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R,
                                                          ss_out, Y, ld, slab, ctr);
}

// the register-streamed short-K projection; 1 = not eligible
template <int KW, int MS, int NM, int EPI, bool BIAS>
int launch_xstream_kw(const GemmCfg &c, hipStream_t s, const uint16_t *X, const uint16_t *W, int m, int n, int k,
                      float eps, const float *ss_in, const uint16_t *Bs, uint16_t *R, float *ss_out, uint16_t *Y,
                      int ld) {
    xstream_gemm_kernel<KW, MS, NM, EPI, BIAS, 0><<<dim3((unsigned)c.gx), 512, 0, s>>>(X, W, m, n, k, eps, ss_in, Bs,
                                                                                    R, ss_out, Y, ld, c.fw, c.xf);
    return launch_status();
}

template <int MS, int NM, int EPI, bool BIAS>
int launch_xstream_ms(const GemmCfg &c, hipStream_t s, const uint16_t *X, const uint16_t *W, int m, int n, int k,
                      float eps, const float *ss_in, const uint16_t *Bs, uint16_t *R, float *ss_out, uint16_t *Y,
                      int ld) {
    const int ks = k / 32, kwn = (ks + 7) / 8;
    if (kwn <= 2) return launch_xstream_kw<2, MS, NM, EPI, BIAS>(c, s, X, W, m, n, k, eps, ss_in, Bs, R, ss_out, Y, ld);
    if (kwn <= 4) return launch_xstream_kw<4, MS, NM, EPI, BIAS>(c, s, X, W, m, n, k, eps, ss_in, Bs, R, ss_out, Y, ld);
    return launch_xstream_kw<8, MS, NM, EPI, BIAS>(c, s, X, W, m, n, k, eps, ss_in, Bs, R, ss_out, Y, ld);
}

int launch_xstream(const GemmCfg &c, hipStream_t s, const uint16_t *X, const uint16_t *W, int m, int n, int k, int nm,
                   float eps, const float *ss_in, const uint16_t *Bs, uint16_t *R, float *ss_out, uint16_t *Y, int ld) {
    const bool lds_image = !launch_policy().xstream;  // policy 0: decode_gemm_kernel's LDS image (A/B)
    const int ks = k / 32;
    if ((lds_image && !c.xf) || c.cb != 1 || c.wn != 1 || c.s != 1 || c.persist || c.nw != 8 || n % 16 ||
        ks < 8 || ks > (c.xf ? 152 : 64) || (c.ms != 1 && c.ms != 2))
        return 1;
    if (R) {  // o_proj: s += x W^T (+ the next norm's partial sums); down_proj over a fragment-order X
        if (nm != 0 || Bs || c.ms != 1) return 1;
        if (c.xf) {
            if (m % 16 || (ks + 7) / 8 > 19) return 1;
            if ((ks + 7) / 8 > 8)
                return launch_xstream_kw<19, 1, 0, EPI_RESIDUAL, false>(c, s, X, W, m, n, k, eps, nullptr, nullptr, R,
                                                                       ss_out, nullptr, ld);
        }
        return launch_xstream_ms<1, 0, EPI_RESIDUAL, false>(c, s, X, W, m, n, k, eps, nullptr, nullptr, R, ss_out, nullptr,
                                                            ld);
    }
    if (c.xf) return 1;
    if (nm != 2 || !ss_in || !Bs || !Y) return 1;  // qkv: folded norm + bias
    if (c.ms == 1)
        return launch_xstream_ms<1, 2, EPI_PLAIN, true>(c, s, X, W, m, n, k, eps, ss_in, Bs, nullptr, nullptr, Y, ld);
    return launch_xstream_ms<2, 2, EPI_PLAIN, true>(c, s, X, W, m, n, k, eps, ss_in, Bs, nullptr, nullptr, Y, ld);
}

template <int MS, int NM, int EPI, bool BIAS>
int launch_gemm_cb(const GemmCfg &c, dim3 grid, size_t lds, hipStream_t s, const uint16_t *X, const uint16_t *W,
                   int m, int n, int k, const uint16_t *NWt, float eps, const float *ss_in, const uint16_t *Bs,
                   uint16_t *R, float *ss_out, uint16_t *Y, int ld, float *slab, int *ctr) {
    switch (c.cb / c.wn) {  // column blocks per wave
    case 1:
        if (c.nw > 8)  // 16 waves: one-column-block tiles over long K
            return launch_gemm<1, MS, NM, EPI, BIAS, 1024>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr);
        return launch_gemm<1, MS, NM, EPI, BIAS, 512>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr);
    case 2: return launch_gemm<2, MS, NM, EPI, BIAS, 512>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr);
    default: return launch_gemm<4, MS, NM, EPI, BIAS, 512>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr);
    }
}

template <int NM, int EPI, bool BIAS>
int launch_gemm_ms(const GemmCfg &c, dim3 grid, size_t lds, hipStream_t s, const uint16_t *X, const uint16_t *W,
                   int m, int n, int k, const uint16_t *NWt, float eps, const float *ss_in, const uint16_t *Bs,
                   uint16_t *R, float *ss_out, uint16_t *Y, int ld, float *slab, int *ctr) {
    switch (c.ms) {
    case 1: return launch_gemm_cb<1, NM, EPI, BIAS>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr);
    case 2: return launch_gemm_cb<2, NM, EPI, BIAS>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr);
    default: return launch_gemm_cb<4, NM, EPI, BIAS>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr);
    }
}

template <int NM, int EPI, bool BIAS, int SAMPLE, int KSC, int RD = 0>
int launch_lm_ks(dim3 grid, size_t lds, hipStream_t s, const uint16_t *X, const uint16_t *W, int M, int N, int K,
                 const uint16_t *NWt, float eps, const float *ss_in, const uint16_t *Bs, uint16_t *Y, int ldy,
                 const LmSample &smp) {
    if (!lds_opt_in<&lm_head_kernel<NM, EPI, BIAS, SAMPLE, KSC, RD>>()) return SWH_E_LAUNCH;  // > 64 KB LDS
    lm_head_kernel<NM, EPI, BIAS, SAMPLE, KSC, RD><<<grid, RD ? 768 : 512, lds, s>>>(X, W, M, N, K, NWt, eps, ss_in, Bs,
                                                                                  Y, ldy, smp);
    return launch_status();
}

// the fused sampler at K = 896 with the half-tile weight ring and 12 waves per workgroup
// (three per SIMD): 58.2-58.8 against 60.3-60.4 us per launch, bench +0.6 % (launch policy
// lm_ring14 = 0: off; read per call)
inline bool lm_ring14() { return launch_policy().lm_ring14 != 0; }

// compile-time k-step counts for the model widths in use (Qwen2.5-0.5B: H = 896)
template <int NM, int EPI, bool BIAS, int SAMPLE>
int launch_lm(dim3 grid, size_t lds, hipStream_t s, const uint16_t *X, const uint16_t *W, int M, int N, int K,
              const uint16_t *NWt, float eps, const float *ss_in, const uint16_t *Bs, uint16_t *Y, int ldy,
              const LmSample &smp) {
    if constexpr (SAMPLE == 1 || SAMPLE == 3) {  // the division instantiation when the rows are sampled at T != 1
        if (!smp.p.greedy && smp.p.temperature != 1.0f)
            return launch_lm<NM, EPI, BIAS, SAMPLE + 1>(grid, lds, s, X, W, M, N, K, NWt, eps, ss_in, Bs, Y, ldy, smp);
    }
    switch (K / 32) {
    case 28:
        if ((SAMPLE == 1 || SAMPLE == 2) && lm_ring14())  // (the log-prob variants spill at 768 threads)
            return launch_lm_ks<NM, EPI, BIAS, SAMPLE, 28, 14>(grid, lds, s, X, W, M, N, K, NWt, eps, ss_in, Bs, Y, ldy,
                                                               smp);
        return launch_lm_ks<NM, EPI, BIAS, SAMPLE, 28>(grid, lds, s, X, W, M, N, K, NWt, eps, ss_in, Bs, Y, ldy, smp);
    case 32: return launch_lm_ks<NM, EPI, BIAS, SAMPLE, 32>(grid, lds, s, X, W, M, N, K, NWt, eps, ss_in, Bs, Y, ldy, smp);
    default: return launch_lm_ks<NM, EPI, BIAS, SAMPLE, 0>(grid, lds, s, X, W, M, N, K, NWt, eps, ss_in, Bs, Y, ldy, smp);
    }
}


// the tile kernel for plain / bias / SiLU epilogues
template <int EPI, bool BIAS>
int launch_tiles(int nm, dim3 grid, size_t lds, hipStream_t s, const uint16_t *X, const uint16_t *W, int M, int N,
                 int K, const uint16_t *NWt, float eps, const float *ss_in, const uint16_t *Bs, uint16_t *Y, int ldy,
                 int fw, int yf = 0) {
    LmSample none{};
    none.fw = fw;
    none.yf = yf;
    if (nm == 1) return launch_lm<1, EPI, BIAS, false>(grid, lds, s, X, W, M, N, K, NWt, eps, ss_in, Bs, Y, ldy, none);
    if (nm == 2) return launch_lm<2, EPI, BIAS, false>(grid, lds, s, X, W, M, N, K, nullptr, eps, ss_in, Bs, Y, ldy, none);
    return launch_lm<0, EPI, BIAS, false>(grid, lds, s, X, W, M, N, K, nullptr, eps, nullptr, Bs, Y, ldy, none);
}

}  // namespace
}  // namespace swh

using namespace swh;

static int attn_decode_impl(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                            const float *rope_sin, const int32_t *prompt_len, const int32_t *prompt_row,
                            const int32_t *state, int64_t B, int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax,
                            float scale, void *out, int32_t out_frag, AttnPrefetch pf, void *stream) {
    if (!qkv || !k_cache || !v_cache || !rope_cos || !rope_sin || !prompt_len || !state || !out || B < 0 || Hkv <= 0 ||
        Hq % Hkv || Tmax <= 0 || B > 65535 || (out_frag & ~1))
        return SWH_E_ARG;
    if (out_frag && (B % 16 || (Hq * D) % 32 || (reinterpret_cast<uintptr_t>(out) & 15))) return SWH_E_ARG;
    if (B == 0) return SWH_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const auto *q = static_cast<const uint16_t *>(qkv);
    auto *kc = static_cast<uint16_t *>(k_cache), *vc = static_cast<uint16_t *>(v_cache);
    auto *o = static_cast<uint16_t *>(out);
    const int gq = Hq / Hkv;
    pf.rows = (int)B;
    pf.prow = prompt_row;
    pf.ofrag = out_frag;
    if (D == 64) return attn_dispatch_gq<64>(gq, q, kc, vc, rope_cos, rope_sin, prompt_len, state, B, Hq, Hkv, Tmax, scale, o, s, pf);
    if (D == 128) return attn_dispatch_gq<128>(gq, q, kc, vc, rope_cos, rope_sin, prompt_len, state, B, Hq, Hkv, Tmax, scale, o, s, pf);
    return SWH_E_ARG;
}

extern "C" int swh_attn_decode_shared_frag(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                                           const float *rope_sin, const int32_t *prompt_len,
                                           const int32_t *prompt_row, const int32_t *state, int64_t B, int32_t Hq,
                                           int32_t Hkv, int32_t D, int32_t Tmax, float scale, void *out,
                                           int32_t out_frag, void *stream) {
    return attn_decode_impl(qkv, k_cache, v_cache, rope_cos, rope_sin, prompt_len, prompt_row, state, B, Hq, Hkv, D,
                            Tmax, scale, out, out_frag, AttnPrefetch{}, stream);
}
// swh_attn_decode_shared_frag whose launch also carries Infinity Cache warm-up
// workgroups (on the CUs the attention leaves idle) over l3_jobs
extern "C" int swh_attn_decode_l3(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                                  const float *rope_sin, const int32_t *prompt_len, const int32_t *prompt_row,
                                  const int32_t *state, int64_t B, int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax,
                                  float scale, void *out, int32_t out_frag, const void *l3_jobs, int32_t l3_njobs,
                                  int32_t l3_wgs, void *l3_sink, void *stream) {
    if (!l3_jobs || !l3_sink || l3_njobs <= 0 || l3_njobs > kL3MaxJobs || l3_wgs <= 0 || l3_wgs > 4096 || Hkv <= 0)
        return SWH_E_ARG;
    AttnPrefetch pf{};
    pf.jobs = static_cast<const L3Job *>(l3_jobs);
    pf.njobs = l3_njobs;
    pf.sink = static_cast<uint32_t *>(l3_sink);
    // the sink holds one word per thread of every warm-up workgroup (whole grid rows)
    pf.nwg = (l3_wgs + Hkv - 1) / Hkv * Hkv;
    return attn_decode_impl(qkv, k_cache, v_cache, rope_cos, rope_sin, prompt_len, prompt_row, state, B, Hq, Hkv, D,
                            Tmax, scale, out, out_frag, pf, stream);
}

extern "C" int swh_attn_decode_shared(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                                      const float *rope_sin, const int32_t *prompt_len, const int32_t *prompt_row,
                                      const int32_t *state, int64_t B, int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax,
                                      float scale, void *out, void *stream) {
    return swh_attn_decode_shared_frag(qkv, k_cache, v_cache, rope_cos, rope_sin, prompt_len, prompt_row, state, B, Hq,
                                       Hkv, D, Tmax, scale, out, 0, stream);
}

extern "C" int swh_attn_decode(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                               const float *rope_sin, const int32_t *prompt_len, const int32_t *state, int64_t B,
                               int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax, float scale, void *out,
                               void *stream) {
    return swh_attn_decode_shared(qkv, k_cache, v_cache, rope_cos, rope_sin, prompt_len, nullptr, state, B, Hq, Hkv, D,
                                  Tmax, scale, out, stream);
}

extern "C" int64_t swh_decode_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
    if (M <= 0 || N <= 0 || K <= 0) return kCounterBytes;
    int64_t a = wide_gemm_slab_bytes(M, N, K, 0), b = wide_gemm_slab_bytes(M, N, K, 1);
    for (int nrm : {0, 1, 2}) {
        const int64_t a1 = slab_bytes(pick_cfg(M, N, K, false, nrm), M, N);
        const int64_t b1 = slab_bytes(pick_cfg(M, 2 * N, K, true, nrm), M, 2 * N);
        a = a1 > a ? a1 : a;
        b = b1 > b ? b1 : b;
    }
    return kCounterBytes + (a > b ? a : b);
}

// fw: W in the swh_frag_pack layout (no norm_w, K % 128 == 0): the wide path
// reads row-major or its own packed weights only, so fw skips it
static int decode_gemm_impl(const void *x, const void *w, int64_t M, int64_t N, int64_t K, const void *norm_w,
                            float eps, const void *bias, void *residual, int32_t silu, void *y, int64_t ldy,
                            const float *ss_in, float *ss_out, void *workspace, int64_t workspace_bytes, void *stream,
                            int fw, int act = 0) {
    if (fw && (norm_w || K % 128)) return SWH_E_ARG;
    // act bit 0: the SiLU output in fragment order (tile path only); bit 1: X in fragment order (xstream only)
    if (act & ~3 || ((act & 1) && (!silu || N % 32 || M % 16)) || ((act & 2) && (!residual || M % 16 || K % 32)))
        return SWH_E_ARG;
    if (!x || !w || M <= 0 || N <= 0 || K <= 0 || K % 64 || M > (1 << 20) || N >= (1 << 29) || K >= (1 << 29))
        return SWH_E_ARG;
    if (residual && (silu || bias)) return SWH_E_ARG;
    if (!residual && !y) return SWH_E_ARG;
    if (ss_in && !norm_w && residual) return SWH_E_ARG;  // folded-norm row scale: plain / SiLU epilogues
    if (ss_out && !residual) return SWH_E_ARG;
    if (N % (silu ? 8 : 16) || ldy % 8 || ldy < N) return SWH_E_ARG;
    const uintptr_t out_ptr = reinterpret_cast<uintptr_t>(residual ? residual : y);
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | out_ptr) & 15) return SWH_E_ARG;
    if ((bias && (reinterpret_cast<uintptr_t>(bias) & 15)) || (norm_w && (reinterpret_cast<uintptr_t>(norm_w) & 15)) ||
        (ss_in && (reinterpret_cast<uintptr_t>(ss_in) & 15)))
        return SWH_E_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t wcols = silu ? 2 * N : N;
    const int nm = norm_w ? 1 : (ss_in ? 2 : 0);
    const swh_launch_policy pol = launch_policy();
    if (!fw && nm != 1 && K >= pol.wide_kmin && pol.wide_gemm) {  // the bandwidth regime (8B decode): csrc/wide_gemm.hip
        const int st = wide_gemm(x, w, M, N, K, eps, ss_in, bias, residual, silu, y, ldy, ss_out, workspace,
                                 workspace_bytes, kCounterBytes, 0, s);
        if (st != 1) return st;
    }
    {  // many 16-column tiles and a K that fits the X image: the tile kernel (lm head, gate/up)
        const int64_t ntile = silu ? N / 8 : N / 16;
        const bool force = pol.gemm_tile != 0, overridden = pol.gemm_ms != 0;  // policy: force / bypass the tile kernel
        // gate/up (SiLU tiles) from one tile per CU up: 11.2 vs 12.4 us at N 9728 (tools/bench_decode.py --ku)
        const int64_t min_tiles = (silu ? 1 : 8) * (int64_t)cu_count();
        // (the epilogues store 8 columns of a row as one 16-B piece: row-major needs ldy % 8 == 0)
        if (!residual && K <= 32 * kLmMaxKS && (force || (!overridden && ntile >= min_tiles)) &&
            ((silu && (act & 1)) || ldy % 8 == 0)) {
            const int64_t nmt = (M + 63) / 64;
            const GemmLds L = gemm_lds(1, 64, 8, (int)K, (int)K, nm, false);
            int64_t per = cu_count() / nmt > 0 ? cu_count() / nmt : 1;
            if (per > ntile) per = ntile;
            const dim3 grid((unsigned)(per * nmt));
            const auto *X = static_cast<const uint16_t *>(x);
            const auto *W = static_cast<const uint16_t *>(w);
            const auto *NWt = static_cast<const uint16_t *>(norm_w);
            const auto *Bs = static_cast<const uint16_t *>(bias);
            auto *Y = static_cast<uint16_t *>(y);
            const size_t lds = (size_t)L.total + (silu ? 8 : 16) * 1024;  // + the epilogue's 1 / 2 KB per wave
            if (silu) return launch_tiles<EPI_SILU, false>(nm, grid, lds, s, X, W, (int)M, (int)N, (int)K, NWt, eps, ss_in, Bs, Y, (int)ldy, fw, act & 1);
            if (Bs) return launch_tiles<EPI_PLAIN, true>(nm, grid, lds, s, X, W, (int)M, (int)N, (int)K, NWt, eps, ss_in, Bs, Y, (int)ldy, fw);
            return launch_tiles<EPI_PLAIN, false>(nm, grid, lds, s, X, W, (int)M, (int)N, (int)K, NWt, eps, ss_in, Bs, Y, (int)ldy, fw);
        }
    }
    if (act & 1) return SWH_E_ARG;  // the fragment-order SiLU output comes from the tile kernel only
    GemmCfg c = pick_cfg(M, wcols, K, silu != 0, nm);
    c.fw = fw;
    c.xf = (act & 2) ? 1 : 0;
    const int64_t MR = 16 * c.ms, nmt = (M + MR - 1) / MR, ncb = wcols / (16 * c.cb);
    // workspace: [counters (zeroed once, self-resetting) | fp32 slabs]
    int *ctr = static_cast<int *>(workspace);
    float *slab = nullptr;
    if (c.s > 1) {
        if (ncb * nmt * (int64_t)sizeof(int) > kCounterBytes) return SWH_E_ARG;
        if (!workspace || workspace_bytes < kCounterBytes + slab_bytes(c, M, wcols)) return SWH_E_ARG;
        // counters live in a FIXED region at the start (never overlapped by any
        // call's slabs, whatever its shape), so a self-reset counter stays zero
        slab = reinterpret_cast<float *>(static_cast<char *>(workspace) + kCounterBytes);
    }
    const auto *X = static_cast<const uint16_t *>(x);
    const auto *W = static_cast<const uint16_t *>(w);
    const auto *NWt = static_cast<const uint16_t *>(norm_w);
    const auto *Bs = static_cast<const uint16_t *>(bias);
    auto *R = static_cast<uint16_t *>(residual);
    auto *Y = static_cast<uint16_t *>(y);
    const int m = (int)M, n = (int)N, k = (int)K, ld = (int)ldy;
    const GemmLds L = gemm_lds(c.cb, (int)MR, c.nw, (int)((K / 32 + c.s - 1) / c.s * 32), (int)K, nm, c.persist,
                               c.wn);
    if (L.total > 160 * 1024 || c.gx <= 0) return SWH_E_ARG;
    const dim3 grid((unsigned)c.gx, 1u, (unsigned)c.s);
    const size_t lds = (size_t)L.total;
#define SWH_GEMM(NORM_, EPI_, BIAS_) \
    return launch_gemm_ms<NORM_, EPI_, BIAS_>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr)
    if (silu) {
        if (nm == 1) SWH_GEMM(1, EPI_SILU, false);
        if (nm == 2) SWH_GEMM(2, EPI_SILU, false);
        SWH_GEMM(0, EPI_SILU, false);
    }
    if (residual) {
        if (nm == 0) {
            const int rc = launch_xstream(c, s, X, W, m, n, k, nm, eps, ss_in, Bs, R, ss_out, nullptr, ld);
            if (rc != 1) return rc;
        }
        if (c.xf) return SWH_E_ARG;  // a fragment-order X is read by xstream only
        if (nm == 1) SWH_GEMM(1, EPI_RESIDUAL, false);
        SWH_GEMM(0, EPI_RESIDUAL, false);
    }
    if (Bs) {
        if (nm == 1) SWH_GEMM(1, EPI_PLAIN, true);
        if (nm == 2) {
            const int rc = launch_xstream(c, s, X, W, m, n, k, nm, eps, ss_in, Bs, nullptr, nullptr, Y, ld);
            if (rc != 1) return rc;
            SWH_GEMM(2, EPI_PLAIN, true);
        }
        SWH_GEMM(0, EPI_PLAIN, true);
    }
    if (nm == 1) SWH_GEMM(1, EPI_PLAIN, false);
    if (nm == 2) SWH_GEMM(2, EPI_PLAIN, false);
    SWH_GEMM(0, EPI_PLAIN, false);
#undef SWH_GEMM
}

extern "C" int swh_decode_gemm(const void *x, const void *w, int64_t M, int64_t N, int64_t K, const void *norm_w,
                               float eps, const void *bias, void *residual, int32_t silu, void *y, int64_t ldy,
                               const float *ss_in, float *ss_out, void *workspace, int64_t workspace_bytes,
                               void *stream) {
    return decode_gemm_impl(x, w, M, N, K, norm_w, eps, bias, residual, silu, y, ldy, ss_in, ss_out, workspace,
                            workspace_bytes, stream, 0);
}

extern "C" int swh_decode_gemm_fragw(const void *x, const void *w, int64_t M, int64_t N, int64_t K, float eps,
                                     const void *bias, void *residual, int32_t silu, void *y, int64_t ldy,
                                     const float *ss_in, float *ss_out, int32_t act_frag, void *workspace,
                                     int64_t workspace_bytes, void *stream) {
    return decode_gemm_impl(x, w, M, N, K, nullptr, eps, bias, residual, silu, y, ldy, ss_in, ss_out, workspace,
                            workspace_bytes, stream, 1, act_frag);
}

extern "C" int swh_frag_pack(const void *w, const void *norm_w, int64_t N, int64_t K, int32_t silu, void *dst,
                             void *stream) {
    const int64_t rows = silu ? 2 * N : N;
    if (!w || !dst || w == dst || N <= 0 || rows % 16 || (silu && N % 8) || K <= 0 || K % 128) return SWH_E_ARG;
    if ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(norm_w)) & 15)
        return SWH_E_ARG;
    return frag_pack(w, norm_w, N, K, silu, dst, static_cast<hipStream_t>(stream));
}

// [partials (M x per x 8 LmPart) | 256 B: the finalize ticket (zero at allocation) |
//  the log-prob variant's (max, sum) partials, M x per x 8 float2]
static int64_t lm_part_bytes(int64_t M, int64_t V = 0) {
    const int64_t nmt = (M + 63) / 64, per = cu_count() / nmt > 0 ? cu_count() / nmt : 1;
    const int64_t wide = V / 256 + 1;  // the wide sampler's partials per row (K > 1024)
    return (M * (per * 8 > wide ? per * 8 : wide) * (int64_t)sizeof(LmPart) + 255) / 256 * 256;
}

extern "C" int64_t swh_lm_head_sample_workspace_bytes(int64_t M, int64_t V, int64_t K) {
    (void)K;
    return 2 * lm_part_bytes(M, V) + 256;  // sizeof(float2) == sizeof(LmPart)
}

static int lm_head_sample_impl(const void *x, const void *w, int64_t M, int64_t V, int64_t K, const void *norm_w,
                               float eps, const float *ss_in, const swh_sample_params *params, const uint64_t *rng,
                               const int32_t *step, int32_t *finished, int64_t *out_tokens, int64_t out_ld,
                               int64_t *cur_tokens, void *workspace, int64_t workspace_bytes, LmNext nx, void *stream,
                               int fw = 0, float *out_logp = nullptr) {
    if (fw && (norm_w || K % 128)) return SWH_E_ARG;  // fragment order: folded weight (ss_in row scale) only
    if (out_logp && fw && K > 32 * kLmMaxKS) return SWH_E_ARG;  // log-probs: the tile kernel (K <= 1024) only
    // K > 1024 (Llama-3-8B): a fragment-order (= wide_pack order) weight through wide_gemm's
    // 256-row tiles with the sampler epilogue, M <= 64, V % 256 == 0
    const bool wide = fw && K > 32 * kLmMaxKS;
    if (!x || !w || !params || !rng || !step || !finished || !out_tokens || !workspace || M <= 0 || V <= 0 ||
        K <= 0 || K % 64 || (K > 32 * kLmMaxKS && !wide) || V % 16 || V >= ((int64_t)1 << 31) || M > (1 << 20))
        return SWH_E_ARG;
    const swh_sample_params p = *params;
    const bool filtered = !p.greedy && ((p.top_k > 0 && p.top_k < V) || p.top_p < 1.0f || p.min_p > 0.f);
    if (filtered || p.repetition_penalty != 1.0f || p.n_eos < 0 || p.n_eos > 4 || !(p.temperature > 0.f))
        return SWH_E_ARG;  // the caller takes logits + swh_sample_step
    if (workspace_bytes < swh_lm_head_sample_workspace_bytes(M, V, K)) return SWH_E_ARG;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w)) & 15) return SWH_E_ARG;
    if ((norm_w && (reinterpret_cast<uintptr_t>(norm_w) & 15)) || (ss_in && (reinterpret_cast<uintptr_t>(ss_in) & 15)))
        return SWH_E_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (wide) {
        int pstride = 0;
        LmPart *part = static_cast<LmPart *>(workspace);
        const int rc = wide_lm_sample(x, w, M, V, K, eps, ss_in, p, rng, step, part, &pstride, s);
        if (rc == 1) return SWH_E_ARG;  // not a wide shape: logits + swh_sample_step
        if (rc != SWH_OK) return rc;
        lm_sample_finalize_kernel<<<dim3((unsigned)M), 256, 0, s>>>(part, pstride, p, step, finished, out_tokens,
                                                                   out_ld, cur_tokens, (int)V, nx);
        return launch_status();
    }
    const int64_t nmt = (M + 63) / 64, per = cu_count() / nmt > 0 ? cu_count() / nmt : 1;
    const int nm = norm_w ? 1 : (ss_in ? 2 : 0);
    const GemmLds L = gemm_lds(1, 64, 8, (int)K, (int)K, nm, false);
    const dim3 grid((unsigned)(per * nmt));
    LmSample smp{p, rng, step, static_cast<LmPart *>(workspace), (int)per, fw};  // one partial per (row, workgroup)
    if (out_logp)
        smp.lpart = reinterpret_cast<float2 *>(static_cast<char *>(workspace) + lm_part_bytes(M, V) + 256);
    const auto *X = static_cast<const uint16_t *>(x);
    const auto *W = static_cast<const uint16_t *>(w);
    const auto *NWt = static_cast<const uint16_t *>(norm_w);
    const size_t lds = (size_t)L.total;
    const int iM = (int)M, iV = (int)V, iK = (int)K;
    int rc;
    if (out_logp)
        rc = nm == 1   ? launch_lm<1, EPI_PLAIN, false, 3>(grid, lds, s, X, W, iM, iV, iK, NWt, eps, ss_in, nullptr, nullptr, 0, smp)
             : nm == 2 ? launch_lm<2, EPI_PLAIN, false, 3>(grid, lds, s, X, W, iM, iV, iK, nullptr, eps, ss_in, nullptr, nullptr, 0, smp)
                       : launch_lm<0, EPI_PLAIN, false, 3>(grid, lds, s, X, W, iM, iV, iK, nullptr, eps, nullptr, nullptr, nullptr, 0, smp);
    else
        rc = nm == 1   ? launch_lm<1, EPI_PLAIN, false, 1>(grid, lds, s, X, W, iM, iV, iK, NWt, eps, ss_in, nullptr, nullptr, 0, smp)
             : nm == 2 ? launch_lm<2, EPI_PLAIN, false, 1>(grid, lds, s, X, W, iM, iV, iK, nullptr, eps, ss_in, nullptr, nullptr, 0, smp)
                       : launch_lm<0, EPI_PLAIN, false, 1>(grid, lds, s, X, W, iM, iV, iK, nullptr, eps, nullptr, nullptr, nullptr, 0, smp);
    if (rc != SWH_OK) return rc;
    lm_sample_finalize_kernel<<<dim3((unsigned)M), 256, 0, s>>>(smp.part, smp.pstride, p, step, finished, out_tokens,
                                                               out_ld, cur_tokens, (int)V, nx, smp.lpart, out_logp, rng);
    return launch_status();
}

// Packed-weight form of the bandwidth-regime decode GEMM (csrc/wide_gemm.hip): w is the
// fragment order swh_wide_pack writes.  Same arguments and epilogues as swh_decode_gemm
// with a folded (or no) norm; shapes wide_gemm does not serve are SWH_E_ARG (no fallback:
// the packed weight has no row-major reading).
extern "C" int swh_wide_gemm_packed(const void *x, const void *w, int64_t M, int64_t N, int64_t K, float eps,
                                    const void *bias, void *residual, int32_t silu, void *y, int64_t ldy,
                                    const float *ss_in, float *ss_out, void *workspace, int64_t workspace_bytes,
                                    void *stream) {
    if (!x || !w || !wide_gemm_eligible(M, N, K, silu)) return SWH_E_ARG;
    if (residual && (silu || bias || ss_in)) return SWH_E_ARG;
    if (!residual && !y) return SWH_E_ARG;
    if (ss_out && !residual) return SWH_E_ARG;
    if (ldy % 8 || ldy < N) return SWH_E_ARG;
    const uintptr_t out_ptr = reinterpret_cast<uintptr_t>(residual ? residual : y);
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | out_ptr) & 15) return SWH_E_ARG;
    if ((bias && (reinterpret_cast<uintptr_t>(bias) & 15)) || (ss_in && (reinterpret_cast<uintptr_t>(ss_in) & 15)))
        return SWH_E_ARG;
    const int st = wide_gemm(x, w, M, N, K, eps, ss_in, bias, residual, silu, y, ldy, ss_out, workspace,
                             workspace_bytes, kCounterBytes, 1, static_cast<hipStream_t>(stream));
    return st == 1 ? SWH_E_ARG : st;
}

// 1 when swh_wide_gemm_packed serves [M rows] x [N (x2 with silu), K].
extern "C" int swh_wide_gemm_eligible(int64_t M, int64_t N, int64_t K, int32_t silu) {
    return wide_gemm_eligible(M, N, K, silu) ? 1 : 0;
}

extern "C" int swh_wide_pack(const void *w, const void *norm_w, int64_t N, int64_t K, int32_t silu, void *dst,
                             void *stream) {
    if (!w || !dst || w == dst) return SWH_E_ARG;
    if ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(dst) |
         reinterpret_cast<uintptr_t>(norm_w)) & 15)
        return SWH_E_ARG;
    return wide_pack(w, norm_w, N, K, silu, dst, static_cast<hipStream_t>(stream));
}

extern "C" int swh_lm_head_sample(const void *x, const void *w, int64_t M, int64_t V, int64_t K, const void *norm_w,
                                  float eps, const float *ss_in, const swh_sample_params *params, const uint64_t *rng,
                                  const int32_t *step, int32_t *finished, int64_t *out_tokens, int64_t out_ld,
                                  int64_t *cur_tokens, void *workspace, int64_t workspace_bytes, void *stream) {
    return lm_head_sample_impl(x, w, M, V, K, norm_w, eps, ss_in, params, rng, step, finished, out_tokens, out_ld,
                               cur_tokens, workspace, workspace_bytes, LmNext{}, stream);
}

static int lm_head_sample_step_impl(const void *x, const void *w, int64_t M, int64_t V, int64_t K,
                                    const void *norm_w, float eps, const float *ss_in,
                                    const swh_sample_params *params, const uint64_t *rng, int32_t *step,
                                    int32_t *finished, int64_t *out_tokens, int64_t out_ld, int64_t *cur_tokens,
                                    const void *embed, void *x_next, float *ss_next, void *workspace,
                                    int64_t workspace_bytes, void *stream, int fw) {
    if (!embed || !x_next || !cur_tokens || K % 16) return SWH_E_ARG;
    if ((reinterpret_cast<uintptr_t>(embed) | reinterpret_cast<uintptr_t>(x_next)) & 15) return SWH_E_ARG;
    if (workspace_bytes < swh_lm_head_sample_workspace_bytes(M, V, K)) return SWH_E_ARG;
    LmNext nx{static_cast<const uint16_t *>(embed), static_cast<uint16_t *>(x_next), ss_next, step,
              reinterpret_cast<int32_t *>(static_cast<char *>(workspace) + lm_part_bytes(M, V)), (int)K, (int)M};
    return lm_head_sample_impl(x, w, M, V, K, norm_w, eps, ss_in, params, rng, step, finished, out_tokens, out_ld,
                               cur_tokens, workspace, workspace_bytes, nx, stream, fw);
}

extern "C" int swh_lm_head_sample_step(const void *x, const void *w, int64_t M, int64_t V, int64_t K,
                                       const void *norm_w, float eps, const float *ss_in,
                                       const swh_sample_params *params, const uint64_t *rng, int32_t *step,
                                       int32_t *finished, int64_t *out_tokens, int64_t out_ld, int64_t *cur_tokens,
                                       const void *embed, void *x_next, float *ss_next, void *workspace,
                                       int64_t workspace_bytes, void *stream) {
    return lm_head_sample_step_impl(x, w, M, V, K, norm_w, eps, ss_in, params, rng, step, finished, out_tokens,
                                    out_ld, cur_tokens, embed, x_next, ss_next, workspace, workspace_bytes, stream, 0);
}

extern "C" int swh_lm_head_sample_fragw(const void *x, const void *w, int64_t M, int64_t V, int64_t K, float eps,
                                        const float *ss_in, const swh_sample_params *params, const uint64_t *rng,
                                        const int32_t *step, int32_t *finished, int64_t *out_tokens, int64_t out_ld,
                                        int64_t *cur_tokens, void *workspace, int64_t workspace_bytes, void *stream) {
    return lm_head_sample_impl(x, w, M, V, K, nullptr, eps, ss_in, params, rng, step, finished, out_tokens, out_ld,
                               cur_tokens, workspace, workspace_bytes, LmNext{}, stream, 1);
}

extern "C" int swh_lm_head_sample_step_fragw(const void *x, const void *w, int64_t M, int64_t V, int64_t K,
                                             float eps, const float *ss_in, const swh_sample_params *params,
                                             const uint64_t *rng, int32_t *step, int32_t *finished,
                                             int64_t *out_tokens, int64_t out_ld, int64_t *cur_tokens,
                                             const void *embed, void *x_next, float *ss_next, void *workspace,
                                             int64_t workspace_bytes, void *stream) {
    return lm_head_sample_step_impl(x, w, M, V, K, nullptr, eps, ss_in, params, rng, step, finished, out_tokens,
                                    out_ld, cur_tokens, embed, x_next, ss_next, workspace, workspace_bytes, stream, 1);
}

// The fused sampler with the drawn token's log-prob under the processed distribution
// (SAMPLE 3 / 4 of lm_head_kernel): one entry for both weight orders, with or without
// the next step's input (embed null: none, the step counter is not advanced).
extern "C" int swh_lm_head_sample_logp(const void *x, const void *w, int64_t M, int64_t V, int64_t K,
                                       const void *norm_w, float eps, const float *ss_in, int32_t frag_weights,
                                       const swh_sample_params *params, const uint64_t *rng, int32_t *step,
                                       int32_t *finished, int64_t *out_tokens, int64_t out_ld, int64_t *cur_tokens,
                                       float *out_logp, const void *embed, void *x_next, float *ss_next,
                                       void *workspace, int64_t workspace_bytes, void *stream) {
    if (!out_logp || (frag_weights & ~1) || K > 32 * kLmMaxKS) return SWH_E_ARG;
    LmNext nx{};
    if (embed) {
        if (!x_next || !cur_tokens || K % 16) return SWH_E_ARG;
        if ((reinterpret_cast<uintptr_t>(embed) | reinterpret_cast<uintptr_t>(x_next)) & 15) return SWH_E_ARG;
        if (workspace_bytes < swh_lm_head_sample_workspace_bytes(M, V, K)) return SWH_E_ARG;
        nx = LmNext{static_cast<const uint16_t *>(embed), static_cast<uint16_t *>(x_next), ss_next, step,
                    reinterpret_cast<int32_t *>(static_cast<char *>(workspace) + lm_part_bytes(M, V)), (int)K, (int)M};
    }
    return lm_head_sample_impl(x, w, M, V, K, norm_w, eps, ss_in, params, rng, step, finished, out_tokens, out_ld,
                               cur_tokens, workspace, workspace_bytes, nx, stream, frag_weights, out_logp);
}
