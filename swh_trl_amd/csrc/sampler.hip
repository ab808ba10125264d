// Rollout sampling step: HF processor chain + exact categorical draw, on device.
//
// Replaces the body of transformers' `GenerationMixin._sample` that the
// reference reaches through grpo_trainer.py:1793-1810 with the
// GenerationConfig of :995-1014 (PPO: ppo_trainer.py:369-375):
//   fp32 scores -> repetition penalty -> min-new-tokens EOS suppression ->
//   temperature -> top-k -> top-p -> min-p -> categorical draw / argmax ->
//   pad-after-EOS bookkeeping.
// The draw is Gumbel-max, argmax_j (z_j - log(-log u_j)), with u_j from a
// Philox4x32-10 stream (key = seed, ctr = {j>>2, row, base+step}); that is an
// exact sample of softmax(z) in one streaming pass, no sort, no cumsum.
//
// Two kernels:
//  * unfiltered rows (no top-k/top-p/min-p): the row is split over S
//    workgroups (B*S >= ~512 WGs fill the chip), each folding its chunk into
//    (max, sum e^{z-m}, best key, best index); `finalize` merges the S partials.
//  * filtered rows: one 1024-thread workgroup per row; thresholds for top-k
//    (count) and top-p (mass) by an 11/11/10-bit radix select in LDS over the
//    order-preserving integer image of z; min-p is the closed form
//    z >= max + ln(min_p).  All three filters keep {z >= tau}, so their
//    composition is the largest tau.
#include "common.hpp"

namespace swh {
namespace {

constexpr int kSplitThreads = 256;
constexpr int kFiltThreads = 1024;
constexpr int kMaxSplit = 64;

struct Partial {
    float m, s1, best;
    int32_t idx;
};

struct Proc {
    float temperature, rep;
    int32_t greedy, suppress, n_eos;
    int32_t eos[4];
    const uint32_t *seen;  // row bitmap or null
    __device__ __forceinline__ float operator()(int64_t j, float x) const {
        float z = x;
        if (seen && ((seen[j >> 5] >> (j & 31)) & 1u)) z = (z < 0.f) ? z * rep : z / rep;
        if (suppress) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e < n_eos && j == eos[e]) z = kNegInf;
        }
        if (!greedy && temperature != 1.0f) z = z / temperature;
        return z;
    }
};

__device__ __forceinline__ Proc make_proc(const swh_sample_params &p, int32_t step, const uint32_t *seen_row) {
    Proc pr;
    pr.temperature = p.temperature;
    pr.rep = p.repetition_penalty;
    pr.greedy = p.greedy;
    pr.suppress = (step < p.min_new_tokens) ? 1 : 0;
    pr.n_eos = p.n_eos;
#pragma unroll
    for (int e = 0; e < 4; ++e) pr.eos[e] = p.eos_ids[e];
    pr.seen = (p.repetition_penalty != 1.0f) ? seen_row : nullptr;
    return pr;
}

// Gumbel noise of element j of row `row`: word (row & 3) of Philox4x32-10 at
// counter {j, row >> 2, ctr_lo, ctr_hi} — one Philox call serves four rows of
// one column (the fused lm-head sampler's C layout holds exactly those).
__device__ __forceinline__ float gumbel_at(uint32_t k0, uint32_t k1, int64_t j, int64_t row, uint64_t ctr_hi) {
    const U4 w = philox4x32_10(U4{(uint32_t)j, (uint32_t)(row >> 2), (uint32_t)ctr_hi, (uint32_t)(ctr_hi >> 32)},
                               k0, k1);
    const int q = (int)(row & 3);
    const uint32_t bits = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
    const float u = u01_from_bits(bits);
    return -fast_log(-fast_log(u));
}

// best-key merge: larger key wins, ties -> smaller index (torch.argmax order)
__device__ __forceinline__ void best_merge(float &bk, int32_t &bi, float k, int32_t i) {
    if (k > bk || (k == bk && (uint32_t)i < (uint32_t)bi)) {
        bk = k;
        bi = i;
    }
}

__device__ __forceinline__ void wave_best(float &bk, int32_t &bi) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float k = __shfl_xor(bk, o, kWave);
        const int32_t i = __shfl_xor(bi, o, kWave);
        best_merge(bk, bi, k, i);
    }
}

// Block reduction of (soft state, best).  red: >= 5 * nwaves floats.
__device__ __forceinline__ void block_partial(SoftState &st, float &bk, int32_t &bi, float *red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    st = wave_soft(st);
    wave_best(bk, bi);
    if (lane == 0) {
        red[wid] = st.m;
        red[nw + wid] = st.s1;
        red[2 * nw + wid] = st.s2;
        red[3 * nw + wid] = bk;
        red[4 * nw + wid] = __int_as_float(bi);
    }
    __syncthreads();
    SoftState r = soft_init();
    float k = kNegInf;
    int32_t i = 0x7fffffff;
    for (int w = 0; w < nw; ++w) {
        r = soft_merge(r, SoftState{red[w], red[nw + w], red[2 * nw + w]});
        best_merge(k, i, red[3 * nw + w], __float_as_int(red[4 * nw + w]));
    }
    __syncthreads();
    st = r;
    bk = k;
    bi = i;
}

// ---------------------------------------------------------------------------
// Unfiltered: split rows.
// ---------------------------------------------------------------------------
template <int DT>
__global__ __launch_bounds__(kSplitThreads) void sample_split_kernel(
    const typename Elem<DT>::T *__restrict__ logits, int64_t V, int64_t ld, swh_sample_params p,
    const uint64_t *__restrict__ rng, const int32_t *__restrict__ step_p, const uint32_t *__restrict__ seen,
    int64_t words, int64_t chunk, Partial *__restrict__ part, float *__restrict__ scores_out) {
    __shared__ float red[5 * (kSplitThreads / kWave)];
    const int64_t b = blockIdx.y;
    const int S = gridDim.x;
    const int s = blockIdx.x;
    const int32_t step = *step_p;
    const Proc pr = make_proc(p, step, seen ? seen + b * words : nullptr);
    const uint64_t seed = rng[0], ctr = rng[1] + (uint64_t)step;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const auto *row = logits + b * ld;
    const int64_t beg = (int64_t)s * chunk;
    const int64_t end = beg + chunk < V ? beg + chunk : V;
    SoftState st = soft_init();
    float bk = kNegInf;
    int32_t bi = 0x7fffffff;
    float *srow = scores_out ? scores_out + b * V : nullptr;
    row_foreach<DT, false>(row, beg, end, threadIdx.x, kSplitThreads, [&](int64_t j, float x) {
        const float z = pr(j, x);
        if (srow) srow[j] = z;
        if (z == kNegInf) return;
        soft_fold<1>(st, &z);
        const float key = p.greedy ? z : z + gumbel_at(k0, k1, j, b, ctr);
        best_merge(bk, bi, key, (int32_t)j);
    });
    block_partial(st, bk, bi, red);
    if (threadIdx.x == 0) part[b * S + s] = Partial{st.m, st.s1, bk, bi};
}

// ---------------------------------------------------------------------------
// Filtered: one workgroup per row, radix-select thresholds.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ord_key(float z) {
    const uint32_t u = __float_as_uint(z);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_to_float(uint32_t k) {
    const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __uint_as_float(u);
}

constexpr int kBins = 2048;

// Block-wide: find the key tau with W(key > tau) < target <= W(key >= tau),
// where W sums weight(z) over elements with z >= lo (the current kept set).
// The bin at each level is the HIGHEST bin whose inclusive suffix weight
// reaches target (a max-reduction, robust to float reassociation).  Returns
// false if the total weight stays below target (keep everything).
template <int DT, typename WF>
__device__ bool radix_select(const typename Elem<DT>::T *row, int64_t V, const Proc &pr, float lo, WF weight,
                             float target, float *hist, float *scan, int *sel, uint32_t &tau_key) {
    uint32_t prefix = 0, pmask = 0;
    float above = 0.f;
    const int t = threadIdx.x;
    const int lane = t & 63, wid = t >> 6, nw = blockDim.x >> 6;
#pragma unroll 1
    for (int lvl = 0; lvl < 3; ++lvl) {
        const int sh = lvl == 0 ? 21 : (lvl == 1 ? 10 : 0);
        const uint32_t dmask = lvl == 2 ? 0x3ffu : 0x7ffu;
        for (int i = t; i < kBins; i += blockDim.x) hist[i] = 0.f;
        if (t == 0) {
            sel[0] = -1;
            sel[1] = kBins;
        }
        __syncthreads();
        row_foreach<DT, false>(row, 0, V, t, blockDim.x, [&](int64_t j, float x) {
            const float z = pr(j, x);
            if (!(z >= lo) || z == kNegInf) return;
            const uint32_t k = ord_key(z);
            if ((k & pmask) != prefix) return;
            atomicAdd(&hist[(k >> sh) & dmask], weight(z));
        });
        __syncthreads();
        const float h0 = hist[2 * t], h1 = hist[2 * t + 1];
        const float tsum = h0 + h1;
        float v = tsum;  // inclusive suffix scan over lanes (higher lanes = higher bins)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const float u = __shfl_down(v, o, kWave);
            if (lane + o < 64) v += u;
        }
        if (lane == 0) scan[wid] = v;
        __syncthreads();
        float after = 0.f;
        for (int w = wid + 1; w < nw; ++w) after += scan[w];
        const float a1 = above + (v - tsum) + after;  // weight strictly above bin 2t+1
        const float a0 = a1 + h1;                     // weight strictly above bin 2t
        int cand = -1;
        if (h1 > 0.f && a1 + h1 >= target) cand = 2 * t + 1;
        else if (h0 > 0.f && a0 + h0 >= target) cand = 2 * t;
        if (cand >= 0) atomicMax(&sel[0], cand);
        if (h0 > 0.f) atomicMin(&sel[1], 2 * t);
        else if (h1 > 0.f) atomicMin(&sel[1], 2 * t + 1);
        __syncthreads();
        int bin = sel[0];
        if (bin < 0) {
            if (lvl == 0) return false;
            bin = sel[1] < kBins ? sel[1] : 0;
        }
        if (bin == 2 * t + 1) scan[nw] = a1;
        if (bin == 2 * t) scan[nw] = a0;
        __syncthreads();
        above = scan[nw];
        __syncthreads();
        prefix |= (uint32_t)bin << sh;
        pmask |= dmask << sh;
    }
    tau_key = prefix;
    return true;
}

template <int DT>
__global__ __launch_bounds__(kFiltThreads) void sample_filtered_kernel(
    const typename Elem<DT>::T *__restrict__ logits, int64_t V, int64_t ld, swh_sample_params p,
    const uint64_t *__restrict__ rng, const int32_t *__restrict__ step_p, const uint32_t *__restrict__ seen,
    int64_t words, Partial *__restrict__ part, float *__restrict__ scores_out) {
    __shared__ float hist[kBins];
    __shared__ float scan[64];
    __shared__ int sel[2];
    __shared__ float red[5 * (kFiltThreads / kWave)];
    const int64_t b = blockIdx.x;
    const int32_t step = *step_p;
    const Proc pr = make_proc(p, step, seen ? seen + b * words : nullptr);
    const auto *row = logits + b * ld;

    // pass 1: max / lse of the processed scores
    SoftState st = soft_init();
    row_foreach<DT, false>(row, 0, V, threadIdx.x, kFiltThreads, [&](int64_t j, float x) {
        const float z = pr(j, x);
        soft_fold<1>(st, &z);
    });
    st = block_soft(st, red);
    const float M = st.m;
    float lo = kNegInf;
    // top-k (count threshold)
    if (p.top_k > 0 && p.top_k < V) {
        uint32_t tk;
        if (radix_select<DT>(row, V, pr, kNegInf, [](float) { return 1.0f; }, (float)p.top_k, hist, scan, sel, tk))
            lo = key_to_float(tk);
    }
    // top-p (mass threshold, renormalised over the top-k survivors)
    if (p.top_p < 1.0f) {
        SoftState sk = soft_init();
        row_foreach<DT, false>(row, 0, V, threadIdx.x, kFiltThreads, [&](int64_t j, float x) {
            float z = pr(j, x);
            if (!(z >= lo)) z = kNegInf;
            soft_fold<1>(sk, &z);
        });
        sk = block_soft(sk, red);
        const float lse_k = sk.m + fast_log(sk.s1);
        uint32_t tp;
        if (radix_select<DT>(row, V, pr, lo, [&](float z) { return fast_exp(z - lse_k); }, p.top_p, hist, scan, sel, tp))
            lo = fmaxf(lo, key_to_float(tp));
    }
    // min-p: p_j < min_p * p_max  <=>  z_j < M + ln(min_p)
    if (p.min_p > 0.f) lo = fmaxf(lo, M + logf(p.min_p));

    // final pass: draw among survivors
    const uint64_t seed = rng[0], ctr = rng[1] + (uint64_t)step;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    SoftState sf = soft_init();
    float bk = kNegInf;
    int32_t bi = 0x7fffffff;
    float *srow = scores_out ? scores_out + b * V : nullptr;
    row_foreach<DT, false>(row, 0, V, threadIdx.x, kFiltThreads, [&](int64_t j, float x) {
        float z = pr(j, x);
        if (!(z >= lo)) z = kNegInf;
        if (srow) srow[j] = z;
        if (z == kNegInf) return;
        soft_fold<1>(sf, &z);
        const float key = z + gumbel_at(k0, k1, j, b, ctr);
        best_merge(bk, bi, key, (int32_t)j);
    });
    block_partial(sf, bk, bi, red);
    if (threadIdx.x == 0) part[b] = Partial{sf.m, sf.s1, bk, bi};
}

// ---------------------------------------------------------------------------
// Finalize: merge partials, log-prob of the pick, EOS / pad bookkeeping.
// ---------------------------------------------------------------------------
template <int DT>
__global__ __launch_bounds__(64) void sample_finalize_kernel(
    const typename Elem<DT>::T *__restrict__ logits, int64_t V, int64_t ld, swh_sample_params p,
    const int32_t *__restrict__ step_p, int S, const Partial *__restrict__ part, int32_t *__restrict__ finished,
    uint32_t *__restrict__ seen, int64_t words, int64_t *__restrict__ out_tokens, int64_t out_ld,
    int64_t *__restrict__ cur_tokens, float *__restrict__ out_logp) {
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int32_t step = *step_p;
    SoftState st = soft_init();
    float bk = kNegInf;
    int32_t bi = 0x7fffffff;
    for (int s = lane; s < S; s += 64) {
        const Partial q = part[b * S + s];
        st = soft_merge(st, SoftState{q.m, q.s1, 0.f});
        best_merge(bk, bi, q.best, q.idx);
    }
    st = wave_soft(st);
    wave_best(bk, bi);
    if (lane != 0) return;
    if (bi < 0 || bi >= V) bi = 0;  // fully masked row (cannot happen with min_tokens_to_keep=1)
    const Proc pr = make_proc(p, step, seen ? seen + b * words : nullptr);
    const float z = pr(bi, Elem<DT>::load(logits + b * ld + bi));
    const float logp = (z - st.m) - fast_log(st.s1);
    int64_t tok = bi;
    const bool was_finished = finished[b] != 0;
    if (p.pad_token_id >= 0 && was_finished) tok = p.pad_token_id;
    bool is_eos = false;
    for (int e = 0; e < p.n_eos && e < 4; ++e) is_eos |= (tok == p.eos_ids[e]);
    if (is_eos) finished[b] = 1;
    out_tokens[b * out_ld + step] = tok;
    if (cur_tokens) cur_tokens[b] = tok;
    if (out_logp) out_logp[b * out_ld + step] = logp;
    if (seen && tok >= 0 && tok < V) seen[b * words + (tok >> 5)] |= 1u << (tok & 31);
}

__global__ void seen_init_kernel(const int64_t *ids, const int32_t *mask, int64_t L, int64_t V, uint32_t *seen,
                                 int64_t words) {
    const int64_t b = blockIdx.x;
    uint32_t *row = seen + b * words;
    for (int64_t w = threadIdx.x; w < words; w += blockDim.x) row[w] = 0u;
    __syncthreads();
    for (int64_t t = threadIdx.x; t < L; t += blockDim.x) {
        const int64_t id = ids[b * L + t];
        if (id < 0 || id >= V) continue;
        if (mask && mask[b * L + t] == 0) continue;
        atomicOr(&row[id >> 5], 1u << (id & 31));
    }
}

__global__ void step_advance_kernel(int32_t *step) { *step += 1; }

int choose_split(int64_t B, int64_t V) {
    int S = 1;
    while (S < kMaxSplit && B * S < 512 && V / (S * 2) >= 2048) S *= 2;
    return S;
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int64_t swh_sample_workspace_bytes(int64_t B, int64_t V) {
    (void)V;
    return B * kMaxSplit * (int64_t)sizeof(Partial);
}

extern "C" int swh_sample_step(const void *logits, int dtype, int64_t B, int64_t V, int64_t ld,
                               const swh_sample_params *params, const uint64_t *rng, const int32_t *step,
                               int32_t *finished, uint32_t *seen, int64_t *out_tokens, int64_t out_ld,
                               int64_t *cur_tokens, float *out_logp, float *scores_out, void *workspace,
                               void *stream) {
    if (!logits || !params || !rng || !step || !finished || !out_tokens || !workspace || B <= 0 || V <= 0 ||
        ld < V || V >= ((int64_t)1 << 31))
        return SWH_E_ARG;
    const swh_sample_params p = *params;
    if (p.n_eos < 0 || p.n_eos > 4 || !(p.temperature > 0.f) || p.top_p <= 0.f || p.top_k < 0) return SWH_E_ARG;
    if (p.repetition_penalty != 1.0f && !seen) return SWH_E_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t words = (V + 31) / 32;
    const bool filtered = !p.greedy && ((p.top_k > 0 && p.top_k < V) || p.top_p < 1.0f || p.min_p > 0.f);
    Partial *part = static_cast<Partial *>(workspace);
    int S = 1;
#define SWH_SAMPLE_LAUNCH(DTC, TY)                                                                              \
    do {                                                                                                        \
        const TY *lg = static_cast<const TY *>(logits);                                                         \
        if (filtered) {                                                                                         \
            sample_filtered_kernel<DTC><<<dim3((unsigned)B), dim3(kFiltThreads), 0, s>>>(lg, V, ld, p, rng, step, \
                                                                                        seen, words, part,       \
                                                                                        scores_out);            \
        } else {                                                                                                \
            S = choose_split(B, V);                                                                             \
            int64_t chunk = (V + S - 1) / S;                                                                    \
            chunk = (chunk + 7) / 8 * 8;                                                                        \
            sample_split_kernel<DTC><<<dim3((unsigned)S, (unsigned)B), dim3(kSplitThreads), 0, s>>>(            \
                lg, V, ld, p, rng, step, seen, words, chunk, part, scores_out);                                 \
        }                                                                                                       \
        sample_finalize_kernel<DTC><<<dim3((unsigned)B), dim3(64), 0, s>>>(lg, V, ld, p, step, S, part,         \
                                                                             finished, seen, words, out_tokens, \
                                                                             out_ld, cur_tokens, out_logp);     \
    } while (0)
    switch (dtype) {
    case SWH_BF16: SWH_SAMPLE_LAUNCH(SWH_BF16, uint16_t); break;
    case SWH_F32: SWH_SAMPLE_LAUNCH(SWH_F32, float); break;
    default: return SWH_E_DTYPE;
    }
#undef SWH_SAMPLE_LAUNCH
    return launch_status();
}

extern "C" int swh_seen_init(const int64_t *ids, const int32_t *mask, int64_t B, int64_t L, int64_t V,
                             uint32_t *seen, void *stream) {
    if (!ids || !seen || B < 0 || L < 0 || V <= 0) return SWH_E_ARG;
    if (B == 0) return SWH_OK;
    seen_init_kernel<<<dim3((unsigned)B), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(ids, mask, L, V, seen,
                                                                                            (V + 31) / 32);
    return launch_status();
}

extern "C" int swh_step_advance(int32_t *step, void *stream) {
    if (!step) return SWH_E_ARG;
    step_advance_kernel<<<1, 1, 0, static_cast<hipStream_t>(stream)>>>(step);
    return launch_status();
}
