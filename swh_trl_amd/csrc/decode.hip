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

#include "common.hpp"

namespace swh {
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

// A fragment of normalised X: bf16(w * bf16(x * rstd)) for 8 consecutive k.
__device__ __forceinline__ uint4 norm_frag(const uint4 &xv, const uint4 &wv, float rs) {
    float x[8], w[8];
    unpack16<SWH_BF16>(xv, x);
    unpack16<SWH_BF16>(wv, w);
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float a = w[2 * k] * round_bf16(x[2 * k] * rs);
        const float b = w[2 * k + 1] * round_bf16(x[2 * k + 1] * rs);
        o[k] = (uint32_t)f32_to_bf16_bits(a) | ((uint32_t)f32_to_bf16_bits(b) << 16);
    }
    return uint4{o[0], o[1], o[2], o[3]};
}

__device__ __forceinline__ uint4 pack8(const float *v) {
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        o[k] = (uint32_t)f32_to_bf16_bits(v[2 * k]) | ((uint32_t)f32_to_bf16_bits(v[2 * k + 1]) << 16);
    return uint4{o[0], o[1], o[2], o[3]};
}


// LDS layout of the GEMM kernel (bytes; host and device compute it alike):
//   [0,256) rstd[64] | [256,272) flag | [512, 512+nwb) norm-weight slice (bf16)
//   | body: RMSNorm partials (phase 1), then the X image [64][Kr*2+16 B];
//     the merge slots [NW/2][64][NB+1] f32 reuse the image, or follow it when
//     the workgroup loops over several column blocks (the image must persist).
struct GemmLds {
    int64_t nw_off, body_off, xs_bytes, slots_off, total;
};
__host__ __device__ inline GemmLds gemm_lds(int cb, int nw, int krmax, bool norm, bool persist) {
    GemmLds L;
    L.nw_off = 512;
    L.body_off = L.nw_off + (norm ? ((int64_t)krmax * 2 + 15) / 16 * 16 : 0);
    L.xs_bytes = (int64_t)kRows * (krmax * 2 + 16);
    const int64_t slots = (int64_t)(nw > 1 ? nw / 2 : 1) * kRows * (16 * cb + 1) * 4;
    const int64_t ssb = norm ? (int64_t)krmax * 4 : 0;  // upper bound of the partials (K <= 4 * threads)
    L.slots_off = L.body_off + (persist ? L.xs_bytes : 0);
    int64_t end = L.body_off + (L.xs_bytes > ssb ? L.xs_bytes : ssb);
    if (L.slots_off + slots > end) end = L.slots_off + slots;
    L.total = end;
    return L;
}

// grid = (column-block slots, M tiles, S k-splits), block = 64*NW threads (NW 4/8).
// A workgroup stages its X slice [64 rows x Kr] into LDS ONCE — full-line 16-B
// loads, RMSNorm applied on the way in — then covers column blocks of NB =
// 16*CB outputs (several when gridDim.x < column blocks: the lm head loops,
// prefetching the next block's weights before merging the current one).
// The NW waves split the slice's k-steps; each issues all weight loads of a
// round of kU k-steps at once (fragment order, nontemporal: read once) and
// takes its A fragments from the LDS image.  Waves merge through a fixed-order
// LDS tree.  S > 1: write-through (sc1) fp32 slabs, an agent-scope ticket, the
// last arriver sums the S slabs in fixed order (deterministic, placement-
// independent — MI355X_MICROARCH.md §Workgroup dispatch) and runs the epilogue.
constexpr int kU = 4;   // k-steps whose loads are issued together
constexpr int kXP = 16; // X pieces (16 B) per thread per staging chunk

template <int CB, bool NORM, int EPI, bool BIAS>
__global__ __launch_bounds__(512) void decode_gemm_kernel(
    const uint16_t *__restrict__ x, const uint16_t *__restrict__ w, int M, int N, int K,
    const uint16_t *__restrict__ norm_w, float eps, const float *__restrict__ ss_in,
    const uint16_t *__restrict__ bias, uint16_t *__restrict__ res, float *__restrict__ ss_out,
    uint16_t *__restrict__ y, int ldy, float *__restrict__ slabs, int *__restrict__ counters) {
    constexpr int NB = 16 * CB, LD = NB + 1;
    constexpr int G8 = (EPI == EPI_SILU) ? CB : NB / 8;  // 8-column output groups per row
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, NT = blockDim.x, NW = NT >> 6;
    const int S = gridDim.z, sidx = blockIdx.z, m0 = blockIdx.y * kRows;
    const int ncb = (EPI == EPI_SILU) ? N / (NB / 2) : N / NB;
    const bool persist = (int)gridDim.x < ncb;
    const int KS = K / 32, kb0 = (int)((int64_t)KS * sidx / S), kb1 = (int)((int64_t)KS * (sidx + 1) / S);
    const int Kr = (kb1 - kb0) * 32, k0 = kb0 * 32, RS = Kr * 2 + 16;
    const GemmLds L = gemm_lds(CB, NW, (KS + S - 1) / S * 32, NORM, persist);
    float *rstd_s = reinterpret_cast<float *>(lds);
    int *flag_s = reinterpret_cast<int *>(lds + 256);
    uint16_t *nw_s = reinterpret_cast<uint16_t *>(lds + L.nw_off);
    unsigned char *xs = lds + L.body_off;
    float *ssp = reinterpret_cast<float *>(lds + L.body_off);
    float *part = reinterpret_cast<float *>(lds + L.slots_off);
    const int rl = lane & 15, kq = (lane >> 4) * 8;
    SWH_GEMM_TRACE(0);

    // ---- (a) RMSNorm partial sums and the norm-weight slice (L2), first in the queue
    const int nc = K / 64;
    const bool use_ss = NORM && ss_in && K <= 4 * NT;
    float4 ssv[4];
    uint4 nwv[2];
    if constexpr (NORM) {
        if (use_ss) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int idx = min(tid + q * NT, kRows * nc - 1);
                const int r = idx / nc, c = idx - r * nc;
                ssv[q] = reinterpret_cast<const float4 *>(ss_in + (int64_t)min(m0 + r, M - 1) * (K / 16))[c];
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q)
            nwv[q] = reinterpret_cast<const uint4 *>(norm_w + k0)[min(tid + q * NT, Kr / 8 - 1)];
    }
    // ---- (b) X slice: 16-B pieces, consecutive lanes along a row (whole lines)
    const int ppr = Kr / 8, npc = kRows * ppr;
    uint4 xv[kXP];
    auto xload = [&](int base) {
#pragma unroll
        for (int j = 0; j < kXP; ++j) {
            const int p = min(base + tid + j * NT, npc - 1);
            const int r = p / ppr, c = p - r * ppr;
            xv[j] = reinterpret_cast<const uint4 *>(x + (int64_t)min(m0 + r, M - 1) * K + k0)[c];
        }
    };
    xload(0);
    // ---- (c) this wave's weights for the first column block (HBM)
    const int ksw0 = kb0 + (kb1 - kb0) * wid / NW, ksw1 = kb0 + (kb1 - kb0) * (wid + 1) / NW;
    const uint16_t *wrow[CB];
    auto set_rows = [&](int n0) {
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            int n;
            if constexpr (EPI == EPI_SILU) {
                const int c = j * 8 + (rl & 7);
                n = (rl < 8) ? n0 + c : N + n0 + c;  // gate rows, then the matching up rows
            } else {
                n = n0 + j * 16 + rl;
            }
            wrow[j] = w + (int64_t)n * K + kq;
        }
    };
    uint4 bv[kU][CB];
    auto issue = [&](int ks) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int kk = max(min(ks + u, ksw1 - 1), 0) * 32;
#pragma unroll
            for (int j = 0; j < CB; ++j) bv[u][j] = ld_nt(reinterpret_cast<const uint4 *>(wrow[j] + kk));
        }
    };
    auto col0 = [&](int cbk) { return cbk * (EPI == EPI_SILU ? NB / 2 : NB); };
    set_rows(col0(blockIdx.x));
    issue(ksw0);
    // epilogue operands of a single-block workgroup (L2): <= 2 per thread in every geometry
    uint4 pre_res[2], pre_bias[2];
    if constexpr (EPI == EPI_RESIDUAL || BIAS) {
        if (!persist) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int idx = min(tid + q * NT, kRows * G8 - 1);
                const int r = idx / G8, gc = col0(blockIdx.x) + (idx - r * G8) * 8;
                if constexpr (EPI == EPI_RESIDUAL)
                    pre_res[q] = *reinterpret_cast<const uint4 *>(res + (int64_t)min(m0 + r, M - 1) * ldy + gc);
                if constexpr (BIAS) pre_bias[q] = *reinterpret_cast<const uint4 *>(bias + gc);
            }
        }
    }
    SWH_GEMM_TRACE(1);

    // ---- (d) row statistic and norm weights into LDS
    if constexpr (NORM) {
        if (use_ss) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int idx = tid + q * NT;
                if (idx < kRows * nc) ssp[idx] = ((ssv[q].x + ssv[q].y) + ssv[q].z) + ssv[q].w;
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (tid + q * NT < Kr / 8) reinterpret_cast<uint4 *>(nw_s)[tid + q * NT] = nwv[q];
        lds_barrier();
        if (use_ss) {
            if (tid < kRows) {
                float ssum = 0.f;
                for (int c = 0; c < nc; ++c) ssum += ssp[tid * nc + c];
                rstd_s[tid] = rsqrtf(ssum / (float)K + eps);
            }
        } else {
            // whole-row pass over X in global memory, one wave per row (coalesced)
            const int nv = K / 8;
            for (int r = wid; r < kRows; r += NW) {
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

    // ---- (e) normalise and write the X image
    auto xstore = [&](int base) {
#pragma unroll
        for (int j = 0; j < kXP; ++j) {
            const int p = base + tid + j * NT;
            if (p < npc) {
                const int r = p / ppr, c = p - r * ppr;
                uint4 v = xv[j];
                if constexpr (NORM) v = norm_frag(v, reinterpret_cast<const uint4 *>(nw_s)[c], rstd_s[r]);
                *reinterpret_cast<uint4 *>(xs + r * RS + c * 16) = v;
            }
        }
    };
    xstore(0);
    for (int base = kXP * NT; base < npc; base += kXP * NT) {
        xload(base);
        xstore(base);
    }
    lds_barrier();
    SWH_GEMM_TRACE(3);

    // ---- (f) column blocks
    auto slot = [&](int s, int r, int c) -> float & { return part[(s * kRows + r) * LD + c]; };
    for (int cbk = blockIdx.x; cbk < ncb; cbk += gridDim.x) {
        const int n0 = col0(cbk);
        f32x4 acc[4][CB];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int ks = ksw0; ks < ksw1; ks += kU) {
            if (ks != ksw0) issue(ks);
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                if (ks + u >= ksw1) break;
                const int kl = ((ks + u - kb0) * 32 + kq) * 2;
                uint4 a[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const uint4 *>(xs + (i * 16 + rl) * RS + kl);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < CB; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[i]), as_bf16x8(bv[u][j]),
                                                                            acc[i][j], 0, 0, 0);
            }
        }
        // the next column block's first weight round overlaps this block's merge
        if (cbk + (int)gridDim.x < ncb) {
            set_rows(col0(cbk + gridDim.x));
            issue(ksw0);
        }
        SWH_GEMM_TRACE(4);

        // ---- merge the NW waves: fixed-order tree through NW/2 LDS slots -> slot 0
        if (!persist) __syncthreads();  // the slots reuse the X image
        auto park = [&](int s) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < CB; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) slot(s, i * 16 + (lane >> 4) * 4 + e, j * 16 + rl) = acc[i][j][e];
        };
        for (int h = NW >> 1; h >= 1; h >>= 1) {
            if (wid >= h && wid < 2 * h) park(wid - h);
            lds_barrier();
            if (wid < h) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < CB; ++j)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            acc[i][j][e] += slot(wid, i * 16 + (lane >> 4) * 4 + e, j * 16 + rl);
            }
            lds_barrier();
        }
        if (wid == 0) park(0);
        lds_barrier();
        SWH_GEMM_TRACE(5);

        // ---- cross-workgroup split-K: publish, ticket, last arriver reduces
        if (S > 1) {
            const int blk = blockIdx.y * ncb + cbk;
            float *my = slabs + ((int64_t)blk * S + sidx) * (kRows * NB);
            for (int idx = tid; idx < kRows * NB; idx += NT)
                __hip_atomic_store(my + idx, slot(0, idx / NB, idx % NB), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                const int t = __hip_atomic_fetch_add(counters + blk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                flag_s[0] = (t == S - 1);
            }
            __syncthreads();
            if (!flag_s[0]) return;  // S > 1 never loops over column blocks
            const float *base = slabs + (int64_t)blk * S * (kRows * NB);
            for (int idx = tid; idx < kRows * NB; idx += NT) {
                float v = 0.f;
                for (int q = 0; q < S; ++q)
                    v += __hip_atomic_load(base + (int64_t)q * kRows * NB + idx, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                slot(0, idx / NB, idx % NB) = v;
            }
            if (tid == 0) __hip_atomic_store(counters + blk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
        }

        // ---- epilogue, 8 output columns (16 B) per thread
        if constexpr (EPI == EPI_SILU) {
            for (int idx = tid; idx < kRows * G8; idx += NT) {
                const int r = idx / G8, jb = idx - r * G8;
                const int gr = m0 + r;
                if (gr >= M) continue;
                float o[8];
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) {
                    const float g = round_bf16(slot(0, r, jb * 16 + cc)), u = round_bf16(slot(0, r, jb * 16 + 8 + cc));
                    o[cc] = round_bf16(g / (1.f + expf(-g))) * u;
                }
                *reinterpret_cast<uint4 *>(y + (int64_t)gr * ldy + n0 + jb * 8) = pack8(o);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int idx = tid + q * NT;
                if (idx >= kRows * G8) break;
                const int r = idx / G8, c8 = (idx - r * G8) * 8;
                const int gr = m0 + r, gc = n0 + c8;
                if (gr >= M) continue;
                float v[8];
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) v[cc] = slot(0, r, c8 + cc);
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
                        slot(0, r, c8 + cc) = sres[cc];
                    }
                    *sp = pack8(sres);
                } else {
                    *reinterpret_cast<uint4 *>(y + (int64_t)gr * ldy + gc) = pack8(v);
                }
            }
            if constexpr (EPI == EPI_RESIDUAL) {
                if (ss_out) {  // partial sums of squares of the new rows, per 16-column chunk
                    __syncthreads();
                    for (int idx = tid; idx < kRows * CB; idx += NT) {
                        const int r = idx / CB, j = idx - r * CB;
                        if (m0 + r >= M) continue;
                        float ss = 0.f;
#pragma unroll
                        for (int cc = 0; cc < 16; ++cc) ss = fmaf(slot(0, r, j * 16 + cc), slot(0, r, j * 16 + cc), ss);
                        ss_out[(int64_t)(m0 + r) * (N / 16) + n0 / 16 + j] = ss;
                    }
                }
            }
        }
        if (persist) __syncthreads();  // slot 0 is rewritten by the next block
    }
    SWH_GEMM_TRACE(6);
}

// ---------------------------------------------------------------------------
// Attention decode (GQA) on MFMA: one workgroup (4 waves) per (kv head,
// sequence).  The GQ query heads of the kv head are the 16 rows (zero-padded)
// of both products: S = Q K^T on v_mfma_f32_16x16x32_bf16 with the cached K
// rows loaded straight into B fragments; online softmax in the C layout (the
// 16 keys of a block sit in 16 lanes); P V on v_mfma_f32_16x16x16_bf16 with P
// and the V block transposed through a per-wave LDS tile.  Waves take
// interleaved 16-key blocks and issue every K/V load of a round before the
// RoPE prologue, so the KV stream is one round trip per 384 (D 64) keys.
// ---------------------------------------------------------------------------
typedef short bf16x4s __attribute__((ext_vector_type(4)));
constexpr int kAttnThreads = 256;
constexpr int kAttnWaves = kAttnThreads / 64;

template <int D, int GQ>
__global__ __launch_bounds__(kAttnThreads) void attn_decode_kernel(
    const uint16_t *__restrict__ qkv, uint16_t *__restrict__ kc, uint16_t *__restrict__ vc,
    const float *__restrict__ rcos, const float *__restrict__ rsin, const int32_t *__restrict__ plen,
    const int32_t *__restrict__ state, int Hq, int Hkv, int Tmax, float scale, uint16_t *__restrict__ out) {
    static_assert(GQ <= 16, "a kv head serves at most 16 query heads");
    constexpr int DC = D / 32;                   // 32-dim chunks: k-steps of Q K^T
    constexpr int DB = D / 16;                   // 16-dim blocks of the output
    constexpr int JB = (D == 64) ? 6 : 3;        // key blocks per wave per round
    constexpr int KPR = JB * 16 * kAttnWaves;    // keys per round
    constexpr int HD = D / 2;
    __shared__ __attribute__((aligned(16))) uint16_t q_s[16 * D];
    __shared__ __attribute__((aligned(16))) uint16_t kn_s[D];
    __shared__ __attribute__((aligned(16))) uint16_t vn_s[D];
    __shared__ __attribute__((aligned(16))) uint16_t pt_s[kAttnWaves][16 * 16];
    __shared__ __attribute__((aligned(16))) uint16_t vt_s[kAttnWaves][16 * D];
    __shared__ float red_s[kAttnWaves][16][D + 2];

    const int kvh = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, c16 = lane & 15;
    // state[0] = index of the token sampled this step; the input token is state[0] - 1
    const int step = state[0] - 1, P = state[1];
    const int pl = plen[b];
    const int slot_new = P + step;
    const int start = P - pl;
    const int pos = pl + step;
    uint16_t *ob = out + b * (int64_t)Hq * D + kvh * GQ * D;
    if (step < 0 || slot_new >= Tmax || pl < 0 || pl > P) {  // never write outside the cache
        for (int idx = tid; idx < GQ * D; idx += kAttnThreads) ob[idx] = 0x7fc0;  // NaN: fail loudly
        return;
    }
    const int n = slot_new - start + 1;  // keys incl. the new one (index n-1)
    const int64_t cbase = (b * Hkv + kvh) * (int64_t)Tmax * D;
    const uint16_t *kb = kc + cbase + (int64_t)start * D + g * 8;
    const uint16_t *vb = vc + cbase + (int64_t)start * D + g * 8;

    u32x4 kr[JB][DC], vr[JB][DC];  // vector types: uint4 structs defeat SROA under selects
#define SWH_ATTN_ISSUE(base_)                                                                  \
    _Pragma("unroll") for (int i = 0; i < JB; ++i) {                                           \
        const int kk = max(min((base_) + (wid + i * kAttnWaves) * 16 + c16, n - 2), 0);        \
        _Pragma("unroll") for (int c = 0; c < DC; ++c) {                                       \
            kr[i][c] = *reinterpret_cast<const u32x4 *>(kb + (int64_t)kk * D + c * 32);        \
            vr[i][c] = *reinterpret_cast<const u32x4 *>(vb + (int64_t)kk * D + c * 32);        \
        }                                                                                      \
    }
    SWH_ATTN_ISSUE(0)  // the KV stream is in flight during RoPE

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
    for (int d = tid; d < D; d += kAttnThreads) {  // KV append (nobody reads the slot from memory this step)
        kc[cbase + (int64_t)slot_new * D + d] = kn_s[d];
        vc[cbase + (int64_t)slot_new * D + d] = vn_s[d];
    }

    u32x4 qa[DC];
#pragma unroll
    for (int c = 0; c < DC; ++c) qa[c] = *reinterpret_cast<const u32x4 *>(q_s + c16 * D + c * 32 + g * 8);
    float m[4], l[4];
    f32x4 o[DB];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = kNegInf;
        l[r] = 0.f;
    }
#pragma unroll
    for (int d = 0; d < DB; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint16_t *pt = pt_s[wid];
    uint16_t *vt = vt_s[wid];

    for (int base = 0; base < n; base += KPR) {
        if (base) {
            SWH_ATTN_ISSUE(base)
        }
        f32x4 sc[JB];
#pragma unroll
        for (int i = 0; i < JB; ++i) {
            const int k0 = base + (wid + i * kAttnWaves) * 16;
            const bool fresh = (k0 + c16 == n - 1);  // the new key/value: from LDS, not the cache
#pragma unroll
            for (int c = 0; c < DC; ++c) {
                const u32x4 kn = *reinterpret_cast<const u32x4 *>(kn_s + c * 32 + g * 8);
                const u32x4 vn = *reinterpret_cast<const u32x4 *>(vn_s + c * 32 + g * 8);
                kr[i][c] = fresh ? kn : kr[i][c];
                vr[i][c] = fresh ? vn : vr[i][c];
            }
            sc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < DC; ++c)
                sc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, qa[c]),
                                                                __builtin_bit_cast(bf16x8, kr[i][c]), sc[i], 0, 0, 0);
            const bool live = k0 + c16 < n;
#pragma unroll
            for (int r = 0; r < 4; ++r) sc[i][r] = live ? sc[i][r] * scale : kNegInf;
        }
        // online softmax: rows = heads 4g+r, a block's 16 keys across the 16 lanes of the group
        float mx[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            mx[r] = m[r];
#pragma unroll
            for (int i = 0; i < JB; ++i) mx[r] = fmaxf(mx[r], sc[i][r]);
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], off, kWave));
            const float corr = (mx[r] == kNegInf) ? 1.f : expf(m[r] - mx[r]);
            l[r] *= corr;
#pragma unroll
            for (int d = 0; d < DB; ++d) o[d][r] *= corr;
            m[r] = mx[r];
#pragma unroll
            for (int i = 0; i < JB; ++i) {
                const float pj = (mx[r] == kNegInf) ? 0.f : expf(sc[i][r] - mx[r]);
                sc[i][r] = pj;
                l[r] += pj;
            }
        }
        // P V, one 16-key block at a time through the wave's LDS tiles
#pragma unroll
        for (int i = 0; i < JB; ++i) {
            const int k0 = base + (wid + i * kAttnWaves) * 16;
            if (k0 < n) {  // wave-uniform
#pragma unroll
                for (int r = 0; r < 4; ++r) pt[(4 * g + r) * 16 + c16] = f32_to_bf16_bits(sc[i][r]);
#pragma unroll
                for (int c = 0; c < DC; ++c) *reinterpret_cast<u32x4 *>(vt + c16 * D + c * 32 + g * 8) = vr[i][c];
                const bf16x4s pa =
                    __builtin_bit_cast(bf16x4s, *reinterpret_cast<const uint2 *>(pt + c16 * 16 + 4 * g));
#pragma unroll
                for (int d = 0; d < DB; ++d) {
                    bf16x4s vbv;
#pragma unroll
                    for (int j = 0; j < 4; ++j) vbv[j] = (short)vt[(4 * g + j) * D + d * 16 + c16];
                    o[d] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pa, vbv, o[d], 0, 0, 0);
                }
            }
        }
    }
    // row sums across the 16 key lanes, then the waves merge through LDS
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) l[r] += __shfl_xor(l[r], off, kWave);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int d = 0; d < DB; ++d) red_s[wid][4 * g + r][d * 16 + c16] = o[d][r];
        if (c16 == 0) {
            red_s[wid][4 * g + r][D] = m[r];
            red_s[wid][4 * g + r][D + 1] = l[r];
        }
    }
    __syncthreads();
    for (int idx = tid; idx < GQ * D; idx += kAttnThreads) {
        const int h = idx / D, d = idx - h * D;
        float mxw = kNegInf;
#pragma unroll
        for (int q = 0; q < kAttnWaves; ++q) mxw = fmaxf(mxw, red_s[q][h][D]);
        float L = 0.f, A = 0.f;
#pragma unroll
        for (int q = 0; q < kAttnWaves; ++q) {
            const float mq = red_s[q][h][D];
            if (mq == kNegInf) continue;
            const float cq = expf(mq - mxw);
            L = fmaf(red_s[q][h][D + 1], cq, L);
            A = fmaf(red_s[q][h][d], cq, A);
        }
        ob[idx] = f32_to_bf16_bits(A / L);
    }
#undef SWH_ATTN_ISSUE
}

template <int D, int GQ>
int launch_attn(const uint16_t *q, uint16_t *kc, uint16_t *vc, const float *rc, const float *rs, const int32_t *pl,
                const int32_t *st, int64_t B, int Hq, int Hkv, int Tmax, float scale, uint16_t *o, hipStream_t s) {
    attn_decode_kernel<D, GQ><<<dim3((unsigned)Hkv, (unsigned)B), kAttnThreads, 0, s>>>(q, kc, vc, rc, rs, pl, st, Hq,
                                                                                      Hkv, Tmax, scale, o);
    return launch_status();
}

template <int D>
int attn_dispatch_gq(int gq, const uint16_t *q, uint16_t *kc, uint16_t *vc, const float *rc, const float *rs,
                     const int32_t *pl, const int32_t *st, int64_t B, int Hq, int Hkv, int Tmax, float scale,
                     uint16_t *o, hipStream_t s) {
    switch (gq) {
    case 1: return launch_attn<D, 1>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 2: return launch_attn<D, 2>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 3: return launch_attn<D, 3>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 4: return launch_attn<D, 4>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 5: return launch_attn<D, 5>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 6: return launch_attn<D, 6>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 7: return launch_attn<D, 7>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 8: return launch_attn<D, 8>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    default: return SWH_E_ARG;
    }
}

// ---- GEMM launch configuration -------------------------------------------
struct GemmCfg {
    int cb, nw, s, gx;  // 16-col blocks per workgroup, waves, K split, grid.x
    bool persist;
};

int cu_count() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

// K slices of <= 1024 (the X image fits LDS); the narrowest column block that
// keeps every workgroup on its own CU; when even 64-column blocks are more
// than the CUs (the lm head) the workgroups loop over column blocks instead.
GemmCfg pick_cfg(int64_t M, int64_t wcols, int64_t K, bool silu) {
    const int64_t mt = (M + kRows - 1) / kRows, KS = K / 32, ncu = cu_count();
    const int64_t align = silu ? 2 : 1;
    GemmCfg c{4, 8, (int)((K + 1023) / 1024), 0, false};
    bool fits = false;
    for (int cb : {1, 2, 4}) {
        if (wcols % (16 * cb * align)) continue;
        if (wcols / (16 * cb) * mt * c.s <= ncu) {
            c.cb = cb;
            fits = true;
            break;
        }
    }
    if (!fits && c.s == 1 && wcols % (32 * align) == 0) {  // persistent over column blocks
        c.cb = 2;
        c.persist = true;
    }
    if (const char *e = getenv("SWH_GEMM_CFG")) {  // tuning override "cb,nw,s"
        int a = 0, b = 0, d = 0;
        if (sscanf(e, "%d,%d,%d", &a, &b, &d) == 3 && (a == 1 || a == 2 || a == 4) && (b == 4 || b == 8) && d >= 1 &&
            d <= KS && wcols % (16 * a * align) == 0 && K / d <= 1024) {
            c.cb = a;
            c.nw = b;
            c.s = d;
            c.persist = (d == 1) && wcols / (16 * a) * mt > ncu;
        }
    }
    const int64_t ncb = wcols / (16 * c.cb);
    c.gx = (int)(c.persist ? (ncu / mt > 0 ? ncu / mt : 1) : ncb);
    if (c.gx > ncb) c.gx = (int)ncb;
    (void)KS;
    return c;
}

int64_t slab_bytes(const GemmCfg &c, int64_t M, int64_t wcols) {
    if (c.s == 1) return 0;
    const int64_t mt = (M + kRows - 1) / kRows;
    return mt * wcols * c.s * kRows * (int64_t)sizeof(float);  // tiles * NB == mt * wcols
}

template <int CB, bool NORM, int EPI, bool BIAS>
int launch_gemm(const GemmCfg &c, dim3 grid, size_t lds, hipStream_t s, const uint16_t *X, const uint16_t *W, int m,
                int n, int k, const uint16_t *NWt, float eps, const float *ss_in, const uint16_t *Bs, uint16_t *R,
                float *ss_out, uint16_t *Y, int ld, float *slab, int *ctr) {
    static bool attr = false;  // > 64 KB of dynamic LDS needs the opt-in once per kernel
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(&decode_gemm_kernel<CB, NORM, EPI, BIAS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return SWH_E_LAUNCH;
        attr = true;
    }
    decode_gemm_kernel<CB, NORM, EPI, BIAS><<<grid, 64u * c.nw, lds, s>>>(X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out,
                                                                         Y, ld, slab, ctr);
    return launch_status();
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int swh_attn_decode(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                               const float *rope_sin, const int32_t *prompt_len, const int32_t *state, int64_t B,
                               int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax, float scale, void *out,
                               void *stream) {
    if (!qkv || !k_cache || !v_cache || !rope_cos || !rope_sin || !prompt_len || !state || !out || B < 0 || Hkv <= 0 ||
        Hq % Hkv || Tmax <= 0 || B > 65535)
        return SWH_E_ARG;
    if (B == 0) return SWH_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const auto *q = static_cast<const uint16_t *>(qkv);
    auto *kc = static_cast<uint16_t *>(k_cache), *vc = static_cast<uint16_t *>(v_cache);
    auto *o = static_cast<uint16_t *>(out);
    const int gq = Hq / Hkv;
    if (D == 64) return attn_dispatch_gq<64>(gq, q, kc, vc, rope_cos, rope_sin, prompt_len, state, B, Hq, Hkv, Tmax, scale, o, s);
    if (D == 128) return attn_dispatch_gq<128>(gq, q, kc, vc, rope_cos, rope_sin, prompt_len, state, B, Hq, Hkv, Tmax, scale, o, s);
    return SWH_E_ARG;
}

extern "C" int64_t swh_decode_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
    if (M <= 0 || N <= 0 || K <= 0) return kCounterBytes;
    const int64_t a = slab_bytes(pick_cfg(M, N, K, false), M, N);
    const int64_t b = slab_bytes(pick_cfg(M, 2 * N, K, true), M, 2 * N);
    return kCounterBytes + (a > b ? a : b);
}

extern "C" int swh_decode_gemm(const void *x, const void *w, int64_t M, int64_t N, int64_t K, const void *norm_w,
                               float eps, const void *bias, void *residual, int32_t silu, void *y, int64_t ldy,
                               const float *ss_in, float *ss_out, void *workspace, int64_t workspace_bytes,
                               void *stream) {
    if (!x || !w || M <= 0 || N <= 0 || K <= 0 || K % 64 || M > (1 << 20) || N >= (1 << 29) || K >= (1 << 29))
        return SWH_E_ARG;
    if (residual && (silu || bias)) return SWH_E_ARG;
    if (!residual && !y) return SWH_E_ARG;
    if (ss_in && !norm_w) return SWH_E_ARG;
    if (ss_out && !residual) return SWH_E_ARG;
    if (N % (silu ? 8 : 16) || ldy % 8 || ldy < N) return SWH_E_ARG;
    const uintptr_t out_ptr = reinterpret_cast<uintptr_t>(residual ? residual : y);
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | out_ptr) & 15) return SWH_E_ARG;
    if ((bias && (reinterpret_cast<uintptr_t>(bias) & 15)) || (norm_w && (reinterpret_cast<uintptr_t>(norm_w) & 15)) ||
        (ss_in && (reinterpret_cast<uintptr_t>(ss_in) & 15)))
        return SWH_E_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t wcols = silu ? 2 * N : N;
    const GemmCfg c = pick_cfg(M, wcols, K, silu != 0);
    const unsigned gy = (unsigned)((M + kRows - 1) / kRows);
    const int64_t blocks = wcols / (16 * c.cb);
    // workspace: [counters (zeroed once, self-resetting) | fp32 slabs]
    int *ctr = static_cast<int *>(workspace);
    float *slab = nullptr;
    if (c.s > 1) {
        if (blocks * gy * (int64_t)sizeof(int) > kCounterBytes) return SWH_E_ARG;
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
    const GemmLds L = gemm_lds(c.cb, c.nw, (int)((K / 32 + c.s - 1) / c.s * 32), NWt != nullptr, c.persist);
    if (L.total > 160 * 1024) return SWH_E_ARG;
    const dim3 grid((unsigned)c.gx, gy, (unsigned)c.s);
    const size_t lds = (size_t)L.total;
#define SWH_GEMM(CB_, NORM_, EPI_, BIAS_) \
    launch_gemm<CB_, NORM_, EPI_, BIAS_>(c, grid, lds, s, X, W, m, n, k, NWt, eps, ss_in, Bs, R, ss_out, Y, ld, slab, ctr)
#define SWH_GEMM_CB(NORM_, EPI_, BIAS_)                                 \
    switch (c.cb) {                                                     \
    case 1: return SWH_GEMM(1, NORM_, EPI_, BIAS_);                     \
    case 2: return SWH_GEMM(2, NORM_, EPI_, BIAS_);                     \
    default: return SWH_GEMM(4, NORM_, EPI_, BIAS_);                    \
    }
    if (silu) {
        if (NWt) SWH_GEMM_CB(true, EPI_SILU, false) else SWH_GEMM_CB(false, EPI_SILU, false)
    } else if (residual) {
        if (NWt) SWH_GEMM_CB(true, EPI_RESIDUAL, false) else SWH_GEMM_CB(false, EPI_RESIDUAL, false)
    } else if (NWt && Bs) {
        SWH_GEMM_CB(true, EPI_PLAIN, true)
    } else if (NWt) {
        SWH_GEMM_CB(true, EPI_PLAIN, false)
    } else if (Bs) {
        SWH_GEMM_CB(false, EPI_PLAIN, true)
    } else {
        SWH_GEMM_CB(false, EPI_PLAIN, false)
    }
#undef SWH_GEMM_CB
#undef SWH_GEMM
}
