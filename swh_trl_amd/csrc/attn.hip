// Causal GQA attention for the full-sequence (training / scoring / prefill)
// forward and backward, bf16 in / out, fp32 softmax statistics.
//
// Replaces torch SDPA in the transformers Qwen2 attention the reference runs
// for every scoring and training forward (grpo_trainer.py:1249 ->
// _get_per_token_logps_and_entropies; the PPO forwards ppo_trainer.py:
// 86-96): at the GRPO shape (64 sequences x 14/2 heads x 384 positions x 64)
// aotriton's flash kernels run ~150 us forward / ~430 us backward per layer.
//
// Orientation (the decode kernel's, csrc/decode.hip attn_decode_kernel): one
// WAVE owns 16 queries and walks the keys in blocks of 32.  S^T = K Q^T on
// v_mfma_f32_16x16x32_bf16 with the 16 queries as the MFMA columns, so each
// lane holds one query and 8 keys: the softmax statistics need two lane
// shuffles, and P^T, packed to bf16 pairs, is the B operand of O^T = V^T P^T
// as it stands; V^T comes from the wave's own LDS tile through
// ds_read_b64_tr_b16 (4 keys x 1 dim per lane).  No workgroup barriers: the
// 4 waves of a workgroup are independent (their K/V reads share the CU's L1).
//
// Backward (FA2 split): delta = rowsum(dO * O); the dQ kernel repeats the
// forward walk (S^T, dP^T = V dO^T, dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T);
// the dK/dV kernel gives a wave 16 KEYS and walks the queries of all the
// heads of its KV group (GQA sum): S = Q K^T with keys as the columns,
// dV^T += dO^T P, dK^T += Q^T dS.
//
// Visibility (transformers' 4-D mask as built in engine/model.py): key k is
// seen by query q iff k <= q and (key_mask[k] or (k == q and q has no valid
// key at or before it)); first_valid[b] = index of the row's first valid key.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace swh {
namespace {

typedef __bf16 bf16x8a __attribute__((ext_vector_type(8)));
typedef float f32x4a __attribute__((ext_vector_type(4)));
typedef float f32x2a __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2a __attribute__((ext_vector_type(2)));
typedef short bf16x4sa __attribute__((ext_vector_type(4)));

constexpr int kFaWaves = 4;
constexpr int kFaThreads = 64 * kFaWaves;

__device__ __forceinline__ bf16x4sa fa_tr16(const uint16_t *p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) bf16x4sa *)(const_cast<uint16_t *>(p)));
}

// An operand indexed [B, H, L, D] (D contiguous) stored as up to two segments:
// rows l < P in segment 0 at sequence index b / div0, rows l >= P in segment 1
// at b / div1, each with its own element strides per sequence, head and row.
// P = 0 is one plain segment.  This is how the GRPO shared-prompt forward
// (engine/model.py hidden_states_grouped) hands over the group's prompt Q/K/V
// once per group and each row's completion, and takes the output token-major
// ([tokens, Hq D], the o_proj input) without any concatenation or transpose.
struct FaView {
    uint16_t *base0, *base1;
    int64_t sb0, sh0, sl0, sb1, sh1, sl1;
    int div0, div1;
};
// the rows of one sequence of a view: the divisions by div happen once per
// workgroup here, not per row (a 32-bit division is ~40 instructions)
struct FaRows {
    uint16_t *p, *c;     // head 0 of the sequence in segment 0 / 1
    int64_t hp, hc;      // head strides
    int64_t sp, sc;      // row strides
    int P;
    __device__ __forceinline__ uint16_t *row(int h, int l) const {
        return l < P ? p + (int64_t)h * hp + (int64_t)l * sp : c + (int64_t)h * hc + (int64_t)(l - P) * sc;
    }
};
__device__ __forceinline__ FaRows fa_rows(const FaView &v, int P, int b) {
    FaRows r;
    r.p = v.base0 + (int64_t)(b / v.div0) * v.sb0;
    r.c = v.base1 + (int64_t)(b / v.div1) * v.sb1;
    r.hp = v.sh0;
    r.hc = v.sh1;
    r.sp = v.sl0;
    r.sc = v.sl1;
    r.P = P;
    return r;
}
__device__ __forceinline__ uint16_t *fa_row(const FaView &v, int P, int b, int h, int l) {
    return fa_rows(v, P, b).row(h, l);
}

struct FaArgs {
    FaView q, k, v, o, dout, dq, dk, dv;
    const int32_t *key_mask;     // [B, L] or null (no padding)
    const int32_t *first_valid;  // [B] or null
    float *lse, *delta;          // [B, Hq, L]
    int B, Hq, Hkv, L;
    int P;                       // rows in segment 0 (0: plain layout)
    int G;                       // > 0: queries l < P of sequences b % G != 0 are not computed (their
                                 // output has no slot: the group's first sequence carries the prompt)
    float scale;
};
// a query that is computed and whose output / gradient exists
__device__ __forceinline__ bool fa_qlive(const FaArgs &a, int b, int q) { return !(a.G && (b % a.G) && q < a.P); }

// Key validity of a 32-key block is a bit mask, bit j = key k0 + j inside the sequence
// and unpadded (a ballot, lanes 32-63 repeating 0-31); a lane's 8 keys of the block are
// k0 + 16 t + 4 g + r (t = 0, 1, r = 0..3): bit 16 t + 4 g + r.
// visibility of key k for query q (transformers' mask): causal, unpadded (kv: the key's
// validity bit), or the query itself when it has no valid key at or before it
__device__ __forceinline__ bool fa_vis(int q, int k, bool kv, int fv) {
    return (k <= q) & (kv | ((k == q) & (q < fv)));
}
// The key-validity words of blocks 0 .. nblk - 1 of sequence b into LDS (nblk <= kFaMaskWords),
// one wave per word: the walk then reads its block's word from LDS instead of waiting on
// a mask load per block.  Visible after the caller's next __syncthreads.
constexpr int kFaMaskWords = 64;  // keys < 2048; longer walks ballot per block (fa_block_bits)
__device__ __forceinline__ uint32_t fa_block_bits(const FaArgs &a, int b, int j, int lane) {
    const int k = 32 * j + (lane & 31);
    const bool v = (k < a.L) && (!a.key_mask || a.key_mask[(int64_t)b * a.L + min(k, a.L - 1)] != 0);
    return (uint32_t)__ballot(v);
}
__device__ __forceinline__ void fa_mask_words(const FaArgs &a, int b, int nblk, uint32_t *words, int wid, int nw,
                                              int lane) {
    if (nblk > kFaMaskWords) return;
    for (int j = wid; j < nblk; j += nw) {
        const uint32_t m = fa_block_bits(a, b, j, lane);
        if (lane == 0) words[j] = m;
    }
}

// scores are carried in log2 units (scale * log2 e folded into one FMA before v_exp_f32)
__device__ __forceinline__ float fa_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// rows [r0, r0 + 32) of a [L, D] slab (clamped) as the two 16-row A fragments of
// one 32-row block: lane (g, c16) <- row r0 + 16 t + c16, dims 32 c + 8 g
template <int D>
__device__ __forceinline__ void fa_load_rows(u32x4 (&r)[2][D / 32], const uint16_t *base, int r0, int L, int c16,
                                             int g) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int row = min(r0 + 16 * t + c16, L - 1);
#pragma unroll
        for (int c = 0; c < D / 32; ++c) r[t][c] = *reinterpret_cast<const u32x4 *>(base + (int64_t)row * D + c * 32 + g * 8);
    }
}

// O^T[d][n] += X^T[d][rows of the block] Y^T[rows][n] where the block's 32 rows
// X [32][D] are parked in the wave's LDS tile and Y^T comes as 8 fp32 values per
// lane (rows 4g..4g+3 of the block's first 16, then of its second 16, column c16):
// the decode kernel's P V step (csrc/decode.hip)
template <int D, int VS>
__device__ __forceinline__ void fa_xty(f32x4a (&o)[D / 16], uint16_t *tile, const u32x4 (&x)[2][D / 32],
                                       const float (&y)[8], int c16, int g) {
#pragma unroll
    for (int c = 0; c < D / 32; ++c) {
        *reinterpret_cast<u32x4 *>(tile + c16 * VS + c * 32 + g * 8) = x[0][c];
        *reinterpret_cast<u32x4 *>(tile + (16 + c16) * VS + c * 32 + g * 8) = x[1][c];
    }
    uint32_t pb[4];
#pragma unroll
    for (int h = 0; h < 4; ++h)
        pb[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2a{y[2 * h], y[2 * h + 1]}, bf16x2a));
    const bf16x8a yb = __builtin_bit_cast(bf16x8a, u32x4{pb[0], pb[1], pb[2], pb[3]});
    const int qq = c16 >> 2, pq = c16 & 3;
#pragma unroll
    for (int d = 0; d < D / 16; ++d) {
        const bf16x4sa lo = fa_tr16(tile + (4 * g + qq) * VS + d * 16 + 4 * pq);
        const bf16x4sa hi = fa_tr16(tile + (16 + 4 * g + qq) * VS + d * 16 + 4 * pq);
        const bf16x8a xa = __builtin_bit_cast(
            bf16x8a, u32x4{__builtin_bit_cast(uint2, lo).x, __builtin_bit_cast(uint2, lo).y,
                           __builtin_bit_cast(uint2, hi).x, __builtin_bit_cast(uint2, hi).y});
        o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, yb, o[d], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the tile is rewritten by the next block
}

template <int D>
__device__ __forceinline__ void fa_copy(u32x4 (&dst)[2][D / 32], const u32x4 (&src)[2][D / 32]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < D / 32; ++c) dst[t][c] = src[t][c];
}

// S^T-like product: out[t][r] = sum_d A[row 16 t + 4 g + r][d] B[col c16][d]
template <int D>
__device__ __forceinline__ void fa_abt(f32x4a (&s)[2], const u32x4 (&a)[2][D / 32], const u32x4 (&bq)[D / 32]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        f32x4a acc = f32x4a{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < D / 32; ++c)
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8a, a[t][c]),
                                                          __builtin_bit_cast(bf16x8a, bq[c]), acc, 0, 0, 0);
        s[t] = acc;
    }
}

template <int D>
constexpr int fa_vs() { return D + (D == 64 ? 8 : 16); }

// X^T Y with the 32-row block X already in a (shared) LDS tile: read-only variant of fa_xty
template <int D, int VS>
__device__ __forceinline__ void fa_xty_shared(f32x4a (&o)[D / 16], const uint16_t *tile, const float (&y)[8],
                                              int c16, int g) {
    uint32_t pb[4];
#pragma unroll
    for (int h = 0; h < 4; ++h)
        pb[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2a{y[2 * h], y[2 * h + 1]}, bf16x2a));
    const bf16x8a yb = __builtin_bit_cast(bf16x8a, u32x4{pb[0], pb[1], pb[2], pb[3]});
    const int qq = c16 >> 2, pq = c16 & 3;
#pragma unroll
    for (int d = 0; d < D / 16; ++d) {
        const bf16x4sa lo = fa_tr16(tile + (4 * g + qq) * VS + d * 16 + 4 * pq);
        const bf16x4sa hi = fa_tr16(tile + (16 + 4 * g + qq) * VS + d * 16 + 4 * pq);
        const bf16x8a xa = __builtin_bit_cast(
            bf16x8a, u32x4{__builtin_bit_cast(uint2, lo).x, __builtin_bit_cast(uint2, lo).y,
                           __builtin_bit_cast(uint2, hi).x, __builtin_bit_cast(uint2, hi).y});
        o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, yb, o[d], 0, 0, 0);
    }
}

// the A fragments of a 32-row block from a shared LDS tile: lane (g, c16) <- row 16 t + c16, dims 32 c + 8 g
template <int D, int VS>
__device__ __forceinline__ void fa_rows_lds(u32x4 (&r)[2][D / 32], const uint16_t *tile, int c16, int g) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < D / 32; ++c)
            r[t][c] = *reinterpret_cast<const u32x4 *>(tile + (16 * t + c16) * VS + c * 32 + g * 8);
}

// cooperative staging of a 32-row block of two [L, D] slabs (K and V) by the whole workgroup:
// global -> registers (issued early) -> LDS (written late)
template <int D>
struct FaStage {
    static constexpr int kPieces = 2 * 32 * D / 8;  // 16-B pieces of the two blocks
    static constexpr int kPer = kPieces / 256;        // per thread (blocks have >= 256 threads)
    u32x4 v[kPer];
};
// rowp(which, row): the row of slab `which` (0: K / Q, 1: V / dO)
template <int D, typename RowP>
__device__ __forceinline__ void fa_stage_load(FaStage<D> &st, RowP rowp, int r0, int L, int tid, int nthr) {
#pragma unroll
    for (int j = 0; j < FaStage<D>::kPer; ++j) {
        // every lane loads (surplus pieces repeat the last one and are not stored): no
        // lane-divergent branch around a load, so the compiler's vmcnt waits stay counted
        // instead of draining every load in flight
        const int pc = min(tid + j * nthr, FaStage<D>::kPieces - 1);
        const int which = pc / (32 * D / 8), rem = pc - which * (32 * D / 8);
        const int row = rem / (D / 8), col = rem - row * (D / 8);
        st.v[j] = *reinterpret_cast<const u32x4 *>(rowp(which, min(r0 + row, L - 1)) + col * 8);
    }
}
template <int D, int VS>
__device__ __forceinline__ void fa_stage_store(const FaStage<D> &st, uint16_t *ktile, uint16_t *vtile, int tid,
                                               int nthr) {
#pragma unroll
    for (int j = 0; j < FaStage<D>::kPer; ++j) {
        const int pc = tid + j * nthr;
        if (pc < FaStage<D>::kPieces) {
            const int which = pc / (32 * D / 8), rem = pc - which * (32 * D / 8);
            const int row = rem / (D / 8), col = rem - row * (D / 8);
            *reinterpret_cast<u32x4 *>((which ? vtile : ktile) + row * VS + col * 8) = st.v[j];
        }
    }
}


#ifndef SWH_FA_REVERSE
#define SWH_FA_REVERSE 0  // forward / dQ: query tiles in reverse (longest first) dispatch order
#endif
#ifndef SWH_FA_PD
#define SWH_FA_PD 1  // 32-row K/V blocks in flight (registers) ahead of the computed one (2-4: more VGPRs, slower)
#endif
#ifndef SWH_FA_PR
#define SWH_FA_PR 2  // dK/dV: rounds (2 x 32 queries) in flight ahead of the round being computed
#endif

#ifndef SWH_FA_FWD_QT
#define SWH_FA_FWD_QT 1  // query tiles per wave in the forward (2: 125 vs 102 us at the bench shape)
#endif

// ---- forward: grid (ceil(L / (16 QT)), Hkv, B); a workgroup = the G = Hq / Hkv query
// heads of one KV head (one wave each) over the same 16 QT queries, so every K/V block
// is staged into LDS once (double-buffered, one barrier per block) for all G heads, and
// each wave's K fragments of a block serve its QT query tiles
template <int D, int QT>
__global__ __launch_bounds__(512) void fa_fwd_kernel(FaArgs a) {
    constexpr int DC = D / 32, DB = D / 16, VS = fa_vs<D>();
    __shared__ __attribute__((aligned(16))) uint16_t kt[2][32 * VS], vt[2][32 * VS];
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int lane = tid & 63, wid = tid >> 6, g = lane >> 4, c16 = lane & 15;
    const int b = blockIdx.z, kvh = blockIdx.y, G = a.Hq / a.Hkv, L = a.L;
    const bool active = wid < G;  // waves past the group's heads only help staging (blocks >= 4 waves)
    const int h = kvh * G + min(wid, G - 1);
#if SWH_FA_REVERSE
    const int q0 = (gridDim.x - 1 - blockIdx.x) * 16 * QT;  // the longest causal walks dispatch first
#else
    const int q0 = blockIdx.x * 16 * QT;
#endif
    if (!fa_qlive(a, b, q0 + 16 * QT - 1)) return;  // the whole tile: prompt queries another sequence carries
    const int fv = a.first_valid ? a.first_valid[b] : 0;
    const FaRows kr_b = fa_rows(a.k, a.P, b), vr_b = fa_rows(a.v, a.P, b), qr_b = fa_rows(a.q, a.P, b);
    auto kvrow = [=](int which, int row) -> const uint16_t * {  // by value: no stack object
        return which ? vr_b.row(kvh, row) : kr_b.row(kvh, row);
    };
    u32x4 qf[QT][DC];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        const int qc = min(q0 + 16 * t + c16, L - 1);  // this lane's query column of tile t
        const uint16_t *qr_ = qr_b.row(h, qc);
#pragma unroll
        for (int c = 0; c < DC; ++c) qf[t][c] = *reinterpret_cast<const u32x4 *>(qr_ + c * 32 + g * 8);
    }
    float m[QT], l[QT];
    f32x4a o[QT][DB];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        m[t] = kNegInf;
        l[t] = 0.f;
#pragma unroll
        for (int d = 0; d < DB; ++d) o[t][d] = f32x4a{0.f, 0.f, 0.f, 0.f};
    }
    const int kend = min(q0 + 16 * QT, L);  // causal: keys < kend
    const float sl2 = a.scale * kLog2e;
    constexpr int PD = SWH_FA_PD;
    const int nblk = (kend + 31) >> 5;
    FaStage<D> ring[PD];  // K/V block j in ring[j % PD] from its load to its LDS store, PD blocks ahead
    __shared__ uint32_t kvw[kFaMaskWords];
    fa_mask_words(a, b, nblk, kvw, wid, nthr >> 6, lane);
    auto load = [=](FaStage<D> &r, int j) { fa_stage_load<D>(r, kvrow, 32 * j, L, tid, nthr); };
    auto put = [&](const FaStage<D> &r, int j) { fa_stage_store<D, VS>(r, kt[j & 1], vt[j & 1], tid, nthr); };
    load(ring[0], 0);
    put(ring[0], 0);
#pragma unroll
    for (int u = 1; u <= PD; ++u) load(ring[u % PD], min(u, nblk - 1));  // past the end: repeats, never stored
    __syncthreads();
    for (int j0 = 0; j0 < nblk; j0 += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            const int j = j0 + u, k0 = 32 * j, buf = j & 1;
            if (j >= nblk) break;
            const uint32_t vm = nblk <= kFaMaskWords ? __builtin_amdgcn_readfirstlane(kvw[j]) : fa_block_bits(a, b, j, lane);
            u32x4 kr[2][DC];
            fa_rows_lds<D, VS>(kr, kt[buf], c16, g);
#pragma unroll
            for (int t = 0; t < QT; ++t) {
                const int qt0 = q0 + 16 * t;
                if (k0 >= qt0 + 16) continue;  // wave-uniform: the whole block is in this tile's future
                f32x4a sc[2];
                fa_abt<D>(sc, kr, qf[t]);
                float sv[8];
                if (k0 + 31 <= qt0 && vm == 0xffffffffu) {  // wave-uniform: every key seen by every query
#pragma unroll
                    for (int e = 0; e < 8; ++e) sv[e] = sc[e >> 2][e & 3];
                } else {
#pragma unroll
                    for (int w = 0; w < 2; ++w)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int kb = 16 * w + 4 * g + r;
                            sv[4 * w + r] = fa_vis(qt0 + c16, k0 + kb, (vm >> kb) & 1u, fv) ? sc[w][r] : kNegInf;
                        }
                }
                float bm = fmaxf(fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3])),
                                 fmaxf(fmaxf(sv[4], sv[5]), fmaxf(sv[6], sv[7])));
                bm = fmaxf(bm, __shfl_xor(bm, 16, kWave));
                bm = fmaxf(bm, __shfl_xor(bm, 32, kWave));
                const float mx = fmaxf(m[t], bm * sl2);  // log2 units
                if (__ballot(mx > m[t])) {  // wave-uniform: rescale only when some query's maximum grew
                    const float corr = mx > m[t] ? fa_exp2(m[t] - mx) : 1.f;
                    l[t] *= corr;
#pragma unroll
                    for (int d = 0; d < DB; ++d) o[t][d] *= corr;
                    m[t] = mx;
                }
                const float nmx = mx == kNegInf ? 0.f : -mx;  // masked scores are -inf: p = 0 either way
                float p[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) p[e] = fa_exp2(fmaf(sv[e], sl2, nmx));
                l[t] += ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
                fa_xty_shared<D, VS>(o[t], vt[buf], p, c16, g);
            }
            if (j + 1 < nblk) put(ring[(u + 1) % PD], j + 1);
            load(ring[(u + 1) % PD], min(j + 1 + PD, nblk - 1));
            __syncthreads();
        }
    }
#pragma unroll
    for (int t = 0; t < QT; ++t) {
        float lt = l[t];
        lt += __shfl_xor(lt, 16, kWave);
        lt += __shfl_xor(lt, 32, kWave);
        const int q = q0 + 16 * t + c16;
        if (active && q < L && fa_qlive(a, b, q)) {
            uint16_t *ob = fa_row(a.o, a.P, b, h, q);
            const float inv = 1.f / lt;
#pragma unroll
            for (int d = 0; d < DB; ++d) {
                const uint32_t lo = (uint32_t)f32_to_bf16_bits(o[t][d][0] * inv) |
                                    ((uint32_t)f32_to_bf16_bits(o[t][d][1] * inv) << 16);
                const uint32_t hi = (uint32_t)f32_to_bf16_bits(o[t][d][2] * inv) |
                                    ((uint32_t)f32_to_bf16_bits(o[t][d][3] * inv) << 16);
                *reinterpret_cast<uint2 *>(ob + d * 16 + 4 * g) = uint2{lo, hi};
            }
            if (g == 0) a.lse[((int64_t)b * a.Hq + h) * L + q] = (m[t] + __log2f(lt)) * kLn2;
        }
    }
}

// ---- backward preprocess: delta[q] = sum_d dO[q][d] O[q][d] (one wave per 4 queries... one thread per query)
template <int D>
__global__ __launch_bounds__(256) void fa_delta_kernel(FaArgs a, int64_t rows) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over [B, Hq, L]
    if (r >= rows) return;
    const int l = (int)(r % a.L), h = (int)((r / a.L) % a.Hq), b = (int)(r / ((int64_t)a.L * a.Hq));
    if (!fa_qlive(a, b, l)) return;  // read by no one
    const uint4 *o = reinterpret_cast<const uint4 *>(fa_row(a.o, a.P, b, h, l));
    const uint4 *d = reinterpret_cast<const uint4 *>(fa_row(a.dout, a.P, b, h, l));
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < D / 8; ++c) {
        float x[8], y[8];
        unpack16<SWH_BF16>(o[c], x);
        unpack16<SWH_BF16>(d[c], y);
#pragma unroll
        for (int j = 0; j < 8; ++j) s = fmaf(x[j], y[j], s);
    }
    a.delta[r] = s;
}

// ---- dQ: the forward walk (K / V blocks shared through LDS by the G query heads)
// with dP^T = V dO^T and dQ^T += K^T dS^T
template <int D>
__global__ __launch_bounds__(512) void fa_dq_kernel(FaArgs a) {
    constexpr int DC = D / 32, DB = D / 16, VS = fa_vs<D>();
    __shared__ __attribute__((aligned(16))) uint16_t kt[2][32 * VS], vt[2][32 * VS];
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int lane = tid & 63, wid = tid >> 6, g = lane >> 4, c16 = lane & 15;
    const int b = blockIdx.z, kvh = blockIdx.y, G = a.Hq / a.Hkv, L = a.L;
    const bool active = wid < G;
    const int h = kvh * G + min(wid, G - 1);
#if SWH_FA_REVERSE
    const int q0 = (gridDim.x - 1 - blockIdx.x) * 16;  // the longest causal walks dispatch first
#else
    const int q0 = blockIdx.x * 16;
#endif
    if (!fa_qlive(a, b, q0 + 15)) return;  // the whole tile: prompt queries another sequence carries
    const int qc = min(q0 + c16, L - 1);
    const int fv = a.first_valid ? a.first_valid[b] : 0;
    const int64_t qrow = ((int64_t)b * a.Hq + h) * L;
    const FaRows kr_b = fa_rows(a.k, a.P, b), vr_b = fa_rows(a.v, a.P, b);
    auto kvrow = [=](int which, int row) -> const uint16_t * {  // by value: no stack object
        return which ? vr_b.row(kvh, row) : kr_b.row(kvh, row);
    };
    u32x4 qf[DC], df[DC];
    {
        const uint16_t *qr_ = fa_row(a.q, a.P, b, h, qc), *dr_ = fa_row(a.dout, a.P, b, h, qc);
#pragma unroll
        for (int c = 0; c < DC; ++c) {
            qf[c] = *reinterpret_cast<const u32x4 *>(qr_ + c * 32 + g * 8);
            df[c] = *reinterpret_cast<const u32x4 *>(dr_ + c * 32 + g * 8);
        }
    }
    const float sl2 = a.scale * kLog2e, nlse2 = -a.lse[qrow + qc] * kLog2e, dl = a.delta[qrow + qc];
    f32x4a acc[DB];
#pragma unroll
    for (int d = 0; d < DB; ++d) acc[d] = f32x4a{0.f, 0.f, 0.f, 0.f};
    const int kend = min(q0 + 16, L);
    constexpr int PD = SWH_FA_PD;
    const int nblk = (kend + 31) >> 5;
    FaStage<D> ring[PD];  // K/V block j in ring[j % PD] from its load to its LDS store, PD blocks ahead
    __shared__ uint32_t kvw[kFaMaskWords];
    fa_mask_words(a, b, nblk, kvw, wid, nthr >> 6, lane);
    auto load = [=](FaStage<D> &r, int j) { fa_stage_load<D>(r, kvrow, 32 * j, L, tid, nthr); };
    auto put = [&](const FaStage<D> &r, int j) { fa_stage_store<D, VS>(r, kt[j & 1], vt[j & 1], tid, nthr); };
    load(ring[0], 0);
    put(ring[0], 0);
#pragma unroll
    for (int u = 1; u <= PD; ++u) load(ring[u % PD], min(u, nblk - 1));  // past the end: repeats, never stored
    __syncthreads();
    for (int j0 = 0; j0 < nblk; j0 += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            const int j = j0 + u, k0 = 32 * j, buf = j & 1;
            if (j >= nblk) break;
            const uint32_t vm = nblk <= kFaMaskWords ? __builtin_amdgcn_readfirstlane(kvw[j]) : fa_block_bits(a, b, j, lane);
            u32x4 kr[2][DC], vr[2][DC];
            fa_rows_lds<D, VS>(kr, kt[buf], c16, g);
            fa_rows_lds<D, VS>(vr, vt[buf], c16, g);
            f32x4a s[2], dp[2];
            fa_abt<D>(s, kr, qf);
            fa_abt<D>(dp, vr, df);
            float ds[8];
            if (k0 + 31 <= q0 && vm == 0xffffffffu) {  // wave-uniform: every key seen by every query
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) ds[4 * t + r] = fa_exp2(fmaf(s[t][r], sl2, nlse2)) * (dp[t][r] - dl);
            } else {
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int kb = 16 * t + 4 * g + r;
                        const float p =
                            fa_vis(q0 + c16, k0 + kb, (vm >> kb) & 1u, fv) ? fa_exp2(fmaf(s[t][r], sl2, nlse2)) : 0.f;
                        ds[4 * t + r] = p * (dp[t][r] - dl);
                    }
            }
            fa_xty_shared<D, VS>(acc, kt[buf], ds, c16, g);
            if (j + 1 < nblk) put(ring[(u + 1) % PD], j + 1);
            load(ring[(u + 1) % PD], min(j + 1 + PD, nblk - 1));
            __syncthreads();
        }
    }
    if (active && q0 + c16 < L && fa_qlive(a, b, q0 + c16)) {
        uint16_t *qb = fa_row(a.dq, a.P, b, h, q0 + c16);
#pragma unroll
        for (int d = 0; d < DB; ++d) {
            const uint32_t lo = (uint32_t)f32_to_bf16_bits(acc[d][0] * a.scale) |
                                ((uint32_t)f32_to_bf16_bits(acc[d][1] * a.scale) << 16);
            const uint32_t hi = (uint32_t)f32_to_bf16_bits(acc[d][2] * a.scale) |
                                ((uint32_t)f32_to_bf16_bits(acc[d][3] * a.scale) << 16);
            *reinterpret_cast<uint2 *>(qb + d * 16 + 4 * g) = uint2{lo, hi};
        }
    }
}

// ---- dK / dV: a workgroup owns 64 keys of one KV head (a wave per 16 keys) and walks
// (query head of the group, 32-query block) rounds; each round's Q and dO blocks and
// their softmax statistics are staged into LDS once (double-buffered, one barrier per
// round) for the 4 key tiles, whose waves read Q / dO fragments and the transposed
// tiles from there.  The GQA head sum stays inside each wave's accumulators.
template <int D>
__global__ __launch_bounds__(256) void fa_dkdv_kernel(FaArgs a) {
    constexpr int DC = D / 32, DB = D / 16, VS = fa_vs<D>();
    constexpr int R = 2;  // 32-query sub-blocks per round: more work per barrier / prefetch
    __shared__ __attribute__((aligned(16))) uint16_t qt[2][R][32 * VS], dt[2][R][32 * VS];
    __shared__ __attribute__((aligned(16))) float lse_s[2][32 * R], del_s[2][32 * R];  // lse_s: -lse log2 e
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int lane = tid & 63, wid = tid >> 6, g = lane >> 4, c16 = lane & 15;
    const int b = blockIdx.z, kvh = blockIdx.y, L = a.L, G = a.Hq / a.Hkv;
    const int kb0 = blockIdx.x * 64, k0w = kb0 + wid * 16;
    const int kc = min(k0w + c16, L - 1);  // this lane's key column
    const int fv = a.first_valid ? a.first_valid[b] : 0;
    const bool kmv = (k0w + c16 < L) && (!a.key_mask || a.key_mask[(int64_t)b * L + kc] != 0);
    const bool kall = __ballot(kmv) == ~0ull;  // every key of the wave inside the sequence and unpadded
    const float sl2 = a.scale * kLog2e;
    u32x4 kf[DC], vf[DC];
    {
        const uint16_t *kr_ = fa_row(a.k, a.P, b, kvh, kc), *vr_ = fa_row(a.v, a.P, b, kvh, kc);
#pragma unroll
        for (int c = 0; c < DC; ++c) {
            kf[c] = *reinterpret_cast<const u32x4 *>(kr_ + c * 32 + g * 8);
            vf[c] = *reinterpret_cast<const u32x4 *>(vr_ + c * 32 + g * 8);
        }
    }
    f32x4a dk[DB], dv[DB];
#pragma unroll
    for (int d = 0; d < DB; ++d) {
        dk[d] = f32x4a{0.f, 0.f, 0.f, 0.f};
        dv[d] = f32x4a{0.f, 0.f, 0.f, 0.f};
    }
    // causal: queries >= the workgroup's first key (and past the prompt when another
    // sequence carries this one's prompt queries)
    const int qstart = fa_qlive(a, b, 0) ? kb0 : max(kb0, a.P);
    const int nb = qstart < L ? (L - qstart + 32 * R - 1) / (32 * R) : 0, nit = G * nb;
    // the prologue below prefetches unconditionally (fixed issue order); with no round
    // (nb == 0: qstart >= L) it must still address valid rows: round 0 of head 0, whose
    // row reads clamp to L - 1 and whose values are never used
    const int nbs = nb > 0 ? nb : 1;
    auto rows_of = [&](int it, int64_t &qrow, int &r0) {
        r0 = qstart + 32 * R * (it % nbs);
        qrow = ((int64_t)b * a.Hq + kvh * G + it / nbs) * L;
    };
    // a round's Q / dO blocks and its rows' lse (threads < 32 R) or delta (< 64 R), in
    // registers from load to LDS store; SWH_FA_PR rounds in flight ahead of the computed one
    struct Round {
        FaStage<D> st[R];
        float sd;
    };
    constexpr int PR = SWH_FA_PR;
    Round ring[PR];  // round it in ring[it % PR]
    const FaRows qr_b = fa_rows(a.q, a.P, b), dr_b = fa_rows(a.dout, a.P, b);
    auto load = [&](Round &rd, int it) {
        int64_t qrow;
        int r0;
        rows_of(it, qrow, r0);
        const int hq = kvh * G + it / nbs;
        auto qdrow = [&](int which, int row) -> const uint16_t * {
            return which ? dr_b.row(hq, row) : qr_b.row(hq, row);
        };
#pragma unroll
        for (int h = 0; h < R; ++h) fa_stage_load<D>(rd.st[h], qdrow, r0 + 32 * h, L, tid, nthr);
        const int si = tid < 32 * R ? tid : min(tid - 32 * R, 32 * R - 1);  // every lane loads (see fa_stage_load)
        rd.sd = (tid < 32 * R ? a.lse : a.delta)[qrow + min(r0 + si, L - 1)];
    };
    auto store = [&](const Round &rd, int buf) {  // staged blocks + the rows' -lse log2 e / delta into LDS
#pragma unroll
        for (int h = 0; h < R; ++h) fa_stage_store<D, VS>(rd.st[h], qt[buf][h], dt[buf][h], tid, nthr);
        if (tid < 32 * R) lse_s[buf][tid] = -rd.sd * kLog2e;
        else if (tid < 64 * R) del_s[buf][tid - 32 * R] = rd.sd;
    };
    if (nit) {
        load(ring[0], 0);
        store(ring[0], 0);
    }
#pragma unroll
    for (int u = 1; u <= PR; ++u) load(ring[u % PR], min(u, max(nit - 1, 0)));  // past the end: repeats
    __syncthreads();
    for (int it0 = 0; it0 < nit; it0 += PR) {
#pragma unroll
    for (int u = 0; u < PR; ++u) {
        const int it = it0 + u, buf = it & 1;
        if (it >= nit) break;
        const int r0 = qstart + 32 * R * (it % nb);
#pragma unroll
        for (int h = 0; h < R; ++h) {
            const int rh = r0 + 32 * h;
            if (rh + 31 >= k0w && rh < L && k0w < L) {  // some query of the block sees some key of this wave
                u32x4 qr[2][DC], dr[2][DC];
                fa_rows_lds<D, VS>(qr, qt[buf][h], c16, g);
                fa_rows_lds<D, VS>(dr, dt[buf][h], c16, g);
                f32x4a s[2], dp[2];
                fa_abt<D>(s, qr, kf);   // S[q = rh + 16 t + 4 g + r][key c16]
                fa_abt<D>(dp, dr, vf);  // dP likewise
                float p[8], ds[8];
                const bool full = rh >= k0w + 15 && rh + 31 < L && kall;  // wave-uniform
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const float4 nl = *reinterpret_cast<const float4 *>(&lse_s[buf][32 * h + 16 * t + 4 * g]);
                    const float4 de = *reinterpret_cast<const float4 *>(&del_s[buf][32 * h + 16 * t + 4 * g]);
                    const float nlv[4] = {nl.x, nl.y, nl.z, nl.w}, dev[4] = {de.x, de.y, de.z, de.w};
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float e = fa_exp2(fmaf(s[t][r], sl2, nlv[r]));
                        if (full) {
                            p[4 * t + r] = e;
                            ds[4 * t + r] = e * (dp[t][r] - dev[r]);
                        } else {
                            const int q = rh + 16 * t + 4 * g + r;
                            const bool vis = (q < L) & fa_vis(q, k0w + c16, kmv, fv) & fa_qlive(a, b, q);
                            p[4 * t + r] = vis ? e : 0.f;
                            ds[4 * t + r] = vis ? e * (dp[t][r] - dev[r]) : 0.f;
                        }
                    }
                }
                fa_xty_shared<D, VS>(dv, dt[buf][h], p, c16, g);
                fa_xty_shared<D, VS>(dk, qt[buf][h], ds, c16, g);
            }
        }
        if (it + 1 < nit) store(ring[(u + 1) % PR], (it + 1) & 1);
        load(ring[(u + 1) % PR], min(it + 1 + PR, nit - 1));
        __syncthreads();
    }
    }
    if (k0w + c16 < L) {
        uint16_t *kb = fa_row(a.dk, a.P, b, kvh, k0w + c16);
        uint16_t *vb = fa_row(a.dv, a.P, b, kvh, k0w + c16);
#pragma unroll
        for (int d = 0; d < DB; ++d) {
            const uint32_t klo = (uint32_t)f32_to_bf16_bits(dk[d][0] * a.scale) |
                                 ((uint32_t)f32_to_bf16_bits(dk[d][1] * a.scale) << 16);
            const uint32_t khi = (uint32_t)f32_to_bf16_bits(dk[d][2] * a.scale) |
                                 ((uint32_t)f32_to_bf16_bits(dk[d][3] * a.scale) << 16);
            *reinterpret_cast<uint2 *>(kb + d * 16 + 4 * g) = uint2{klo, khi};
            const uint32_t vlo = (uint32_t)f32_to_bf16_bits(dv[d][0]) | ((uint32_t)f32_to_bf16_bits(dv[d][1]) << 16);
            const uint32_t vhi = (uint32_t)f32_to_bf16_bits(dv[d][2]) | ((uint32_t)f32_to_bf16_bits(dv[d][3]) << 16);
            *reinterpret_cast<uint2 *>(vb + d * 16 + 4 * g) = uint2{vlo, vhi};
        }
    }
}


}  // namespace
}  // namespace swh

using namespace swh;

namespace {
FaView fa_view_of(const swh_attn_view &v) {
    FaView f;
    f.base0 = static_cast<uint16_t *>(v.base[0]);
    f.base1 = static_cast<uint16_t *>(v.base[1]);
    f.sb0 = v.sb[0];
    f.sh0 = v.sh[0];
    f.sl0 = v.sl[0];
    f.sb1 = v.sb[1];
    f.sh1 = v.sh[1];
    f.sl1 = v.sl[1];
    f.div0 = v.div[0];
    f.div1 = v.div[1];
    return f;
}
bool fa_view_ok(const swh_attn_view *v, int64_t P) {
    return v && v->base[1] && v->div[1] >= 1 && (P == 0 || (v->base[0] && v->div[0] >= 1)) &&
           ((reinterpret_cast<uintptr_t>(v->base[0]) | reinterpret_cast<uintptr_t>(v->base[1])) & 15) == 0 &&
           ((v->sb[0] | v->sh[0] | v->sl[0] | v->sb[1] | v->sh[1] | v->sl[1]) & 7) == 0;
}
// the plain [B, H, L, D] layout as a view
swh_attn_view fa_plain(const void *p, int64_t H, int64_t L, int32_t D) {
    swh_attn_view v{};
    v.base[1] = const_cast<void *>(p);
    v.sb[1] = H * L * D;
    v.sh[1] = L * D;
    v.sl[1] = D;
    v.div[0] = v.div[1] = 1;
    return v;
}
bool fa_dims_ok(int64_t B, int32_t Hq, int32_t Hkv, int64_t L, int64_t P, int32_t G, int32_t D) {
    return B > 0 && Hq > 0 && Hkv > 0 && Hq % Hkv == 0 && L > 0 && L <= (1 << 20) && B <= 65535 &&
           Hq / Hkv <= 8 && (D == 64 || D == 128) && P >= 0 && P <= L && G >= 0 && (G == 0 || P > 0);
}
}  // namespace

extern "C" int swh_attn_fwd_v(const swh_attn_view *q, const swh_attn_view *k, const swh_attn_view *v,
                              const swh_attn_view *out, int64_t B, int32_t Hq, int32_t Hkv, int64_t L, int64_t P,
                              int32_t G, int32_t D, float scale, const int32_t *key_mask, const int32_t *first_valid,
                              float *lse, void *stream) {
    if (!fa_dims_ok(B, Hq, Hkv, L, P, G, D) || !fa_view_ok(q, P) || !fa_view_ok(k, P) || !fa_view_ok(v, P) ||
        !fa_view_ok(out, P) || !lse || (!key_mask != !first_valid))
        return SWH_E_ARG;
    FaArgs a{};
    a.q = fa_view_of(*q);
    a.k = fa_view_of(*k);
    a.v = fa_view_of(*v);
    a.o = fa_view_of(*out);
    a.key_mask = key_mask;
    a.first_valid = first_valid;
    a.lse = lse;
    a.B = (int)B;
    a.Hq = Hq;
    a.Hkv = Hkv;
    a.L = (int)L;
    a.P = (int)P;
    a.G = G;
    a.scale = scale;
    const unsigned thr = 64u * (unsigned)(Hq / Hkv < 4 ? 4 : Hq / Hkv);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // SWH_FA_FWD_QT 16-query tiles per wave (the K fragments of a block serve them all)
    constexpr int QT = SWH_FA_FWD_QT;
    const dim3 gq((unsigned)((L + 16 * QT - 1) / (16 * QT)), (unsigned)Hkv, (unsigned)B);
    if (D == 64) fa_fwd_kernel<64, QT><<<gq, thr, 0, s>>>(a);
    else fa_fwd_kernel<128, QT><<<gq, thr, 0, s>>>(a);
    return launch_status();
}

extern "C" int swh_attn_bwd_v_parts(const swh_attn_view *q, const swh_attn_view *k, const swh_attn_view *v,
                                    const swh_attn_view *out, const swh_attn_view *dout, const float *lse, int64_t B,
                                    int32_t Hq, int32_t Hkv, int64_t L, int64_t P, int32_t G, int32_t D, float scale,
                                    const int32_t *key_mask, const int32_t *first_valid, float *delta,
                                    const swh_attn_view *dq, const swh_attn_view *dk, const swh_attn_view *dv,
                                    int32_t parts, void *stream) {
    if (!fa_dims_ok(B, Hq, Hkv, L, P, G, D) || !fa_view_ok(q, P) || !fa_view_ok(k, P) || !fa_view_ok(v, P) ||
        !fa_view_ok(out, P) || !fa_view_ok(dout, P) || !fa_view_ok(dq, P) || !fa_view_ok(dk, P) ||
        !fa_view_ok(dv, P) || !lse || !delta || (!key_mask != !first_valid) || parts <= 0 || parts > 7)
        return SWH_E_ARG;
    FaArgs a{};
    a.q = fa_view_of(*q);
    a.k = fa_view_of(*k);
    a.v = fa_view_of(*v);
    a.o = fa_view_of(*out);
    a.dout = fa_view_of(*dout);
    a.dq = fa_view_of(*dq);
    a.dk = fa_view_of(*dk);
    a.dv = fa_view_of(*dv);
    a.key_mask = key_mask;
    a.first_valid = first_valid;
    a.lse = const_cast<float *>(lse);
    a.delta = delta;
    a.B = (int)B;
    a.Hq = Hq;
    a.Hkv = Hkv;
    a.L = (int)L;
    a.P = (int)P;
    a.G = G;
    a.scale = scale;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t rows = B * Hq * L;
    const dim3 grid((unsigned)((L + 15) / 16), (unsigned)Hkv, (unsigned)B);
    const unsigned thr = 64u * (unsigned)(Hq / Hkv < 4 ? 4 : Hq / Hkv);
    const dim3 gk((unsigned)((L + 63) / 64), (unsigned)Hkv, (unsigned)B);
    const dim3 gd((unsigned)((rows + 255) / 256));
    if (D == 64) {
        if (parts & SWH_ATTN_BWD_DELTA) fa_delta_kernel<64><<<gd, 256, 0, s>>>(a, rows);
        if (parts & SWH_ATTN_BWD_DQ) fa_dq_kernel<64><<<grid, thr, 0, s>>>(a);
        if (parts & SWH_ATTN_BWD_DKDV) fa_dkdv_kernel<64><<<gk, 256, 0, s>>>(a);
    } else {
        if (parts & SWH_ATTN_BWD_DELTA) fa_delta_kernel<128><<<gd, 256, 0, s>>>(a, rows);
        if (parts & SWH_ATTN_BWD_DQ) fa_dq_kernel<128><<<grid, thr, 0, s>>>(a);
        if (parts & SWH_ATTN_BWD_DKDV) fa_dkdv_kernel<128><<<gk, 256, 0, s>>>(a);
    }
    return launch_status();
}

extern "C" int swh_attn_fwd(const void *q, const void *k, const void *v, int64_t B, int32_t Hq, int32_t Hkv,
                            int64_t L, int32_t D, float scale, const int32_t *key_mask, const int32_t *first_valid,
                            void *out, float *lse, void *stream) {
    if (!q || !k || !v || !out) return SWH_E_ARG;
    const swh_attn_view vq = fa_plain(q, Hq, L, D), vk = fa_plain(k, Hkv, L, D), vv = fa_plain(v, Hkv, L, D),
                        vo = fa_plain(out, Hq, L, D);
    return swh_attn_fwd_v(&vq, &vk, &vv, &vo, B, Hq, Hkv, L, 0, 0, D, scale, key_mask, first_valid, lse, stream);
}

extern "C" int swh_attn_bwd_parts(const void *q, const void *k, const void *v, const void *out, const void *dout,
                                  const float *lse, int64_t B, int32_t Hq, int32_t Hkv, int64_t L, int32_t D,
                                  float scale, const int32_t *key_mask, const int32_t *first_valid, float *delta,
                                  void *dq, void *dk, void *dv, int32_t parts, void *stream) {
    if (!q || !k || !v || !out || !dout || !dq || !dk || !dv) return SWH_E_ARG;
    const swh_attn_view vq = fa_plain(q, Hq, L, D), vk = fa_plain(k, Hkv, L, D), vv = fa_plain(v, Hkv, L, D),
                        vo = fa_plain(out, Hq, L, D), vd = fa_plain(dout, Hq, L, D), vdq = fa_plain(dq, Hq, L, D),
                        vdk = fa_plain(dk, Hkv, L, D), vdv = fa_plain(dv, Hkv, L, D);
    return swh_attn_bwd_v_parts(&vq, &vk, &vv, &vo, &vd, lse, B, Hq, Hkv, L, 0, 0, D, scale, key_mask, first_valid,
                                delta, &vdq, &vdk, &vdv, parts, stream);
}

extern "C" int swh_attn_bwd(const void *q, const void *k, const void *v, const void *out, const void *dout,
                            const float *lse, int64_t B, int32_t Hq, int32_t Hkv, int64_t L, int32_t D, float scale,
                            const int32_t *key_mask, const int32_t *first_valid, float *delta, void *dq, void *dk,
                            void *dv, void *stream) {
    return swh_attn_bwd_parts(q, k, v, out, dout, lse, B, Hq, Hkv, L, D, scale, key_mask, first_valid, delta, dq, dk,
                              dv, SWH_ATTN_BWD_DELTA | SWH_ATTN_BWD_DQ | SWH_ATTN_BWD_DKDV, stream);
}
