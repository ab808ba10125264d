// Rollout sampling step: HF processor chain + exact categorical draw, on device.
//
// Replaces the body of transformers' `GenerationMixin._sample` that the
// reference reaches through grpo_trainer.py:1793-1810 with the
// GenerationConfig of :995-1014 (PPO: ppo_trainer.py:369-375):
//   fp32 scores -> repetition penalty -> min-new-tokens EOS suppression ->
//   temperature -> top-k -> top-p -> min-p -> categorical draw / argmax ->
//   pad-after-EOS bookkeeping.
// The draw is Gumbel-max, argmax_j (z_j - log(-log u_j)), with u_j from a
// Philox4x32-10 stream (key = seed, ctr = {j, row >> 2, base + step}, word row & 3);
// that is an exact sample of softmax(z) in one streaming pass, no sort, no cumsum.
// The unfiltered and the general filtered draw passes take four rows per
// workgroup, so one Philox call serves the four rows of a column.
//
// Two kernels:
//  * unfiltered rows (no top-k/top-p/min-p): the row is split over S
//    workgroups (B*S >= ~512 WGs fill the chip), each folding its chunk into
//    (max, sum e^{z-m}, best key, best index); `finalize` merges the S partials.
//  * filtered rows: the same split over workgroups for every pass; thresholds
//    for top-k (count) and top-p (mass) by an 11/11/10-bit radix select over
//    the order-preserving integer image of z (per-split digit histograms, one
//    select launch per digit); min-p is the closed form z >= max + ln(min_p).
//    All three filters keep {z >= tau}, so their composition is the largest tau.
#include <cstdlib>

#include "common.hpp"

namespace swh {
namespace {

constexpr int kSplitThreads = 256;
constexpr int kFiltThreads = 1024;
constexpr int kMaxSplit = 64;       // row splits of the soft / digit passes
constexpr int kMaxDrawSplit = 256;  // splits per row quad of the draw passes (partials per row)
constexpr int kDrawWgs = 1024;      // draw-pass workgroups aimed at (row quads x splits; 512-2048 measured)

struct Partial {
    float m, s1, best;
    int32_t idx;
};

struct Proc {
    float temperature, rep;
    int32_t greedy, suppress, n_eos;
    int32_t eos[4];
    const uint32_t *seen;  // row bitmap or null
    __device__ __forceinline__ float operator()(int64_t j, float x) const { return at(j, x, seen); }
    // the same processing with another row's bitmap (the four-row draw passes)
    __device__ __forceinline__ float at(int64_t j, float x, const uint32_t *sn) const {
        float z = x;
        if (sn && ((sn[j >> 5] >> (j & 31)) & 1u)) z = (z < 0.f) ? z * rep : z / rep;
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
    return gumbel_from_bits(bits);
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

// The draw passes visit four rows (a row quad 4 q .. 4 q + 3) per workgroup: one
// Philox4x32-10 call at counter {j, q, ctr} yields the Gumbel words of column j for
// all four rows (word i: row 4 q + i, the stream gumbel_at defines), a quarter of the
// per-element Philox work of one row per workgroup.  f(j, x[4]) gets the four rows'
// values of column j; rows past B repeat row B - 1 (their results are not written).
template <int DT, typename F>
__device__ __forceinline__ void row4_foreach(const typename Elem<DT>::T *logits, int64_t ld, int64_t b0, int64_t B,
                                             int64_t begin, int64_t end, int tid, int nthreads, F &&f) {
    using T = typename Elem<DT>::T;
    constexpr int PV = kPerVec<DT>;
    if (end <= begin) return;
    const T *rw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) rw[i] = logits + (b0 + i < B ? b0 + i : B - 1) * ld;
    const uintptr_t a = reinterpret_cast<uintptr_t>(rw[0] + begin);
    const bool vec = ((ld * (int64_t)sizeof(T)) & 15) == 0 && (a & (sizeof(T) - 1)) == 0;  // rows share alignment
    int64_t head = vec ? (int64_t)(((16 - (a & 15)) & 15) / sizeof(T)) : end - begin;
    if (head > end - begin) head = end - begin;
    float x[4];
    for (int64_t j = begin + tid; j < begin + head; j += nthreads) {
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = Elem<DT>::load(rw[i] + j);
        f(j, x);
    }
    const int64_t bv = begin + head;
    const int64_t nvec = vec ? (end - bv) / PV : 0;
    auto body = [&](const uint4 (&raw)[4], int64_t j0) {
        float xs[4][PV];
#pragma unroll
        for (int i = 0; i < 4; ++i) unpack16<DT>(raw[i], xs[i]);
#pragma unroll
        for (int k = 0; k < PV; ++k) {
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = xs[i][k];
            f(j0 + k, x);
        }
    };
    // one vector of each of the four rows per trip (four loads in flight): the body is
    // instantiated PV times only — an unrolled second vector doubled the kernel past the
    // instruction cache
    for (int64_t v = tid; v < nvec; v += nthreads) {
        uint4 raw[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) raw[i] = reinterpret_cast<const uint4 *>(rw[i] + bv)[v];
        body(raw, bv + v * PV);
    }
    for (int64_t j = bv + nvec * PV + tid; j < end; j += nthreads) {
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = Elem<DT>::load(rw[i] + j);
        f(j, x);
    }
}

__device__ __forceinline__ void philox_col(uint32_t k0, uint32_t k1, int64_t j, int64_t quad, uint64_t ctr,
                                           uint32_t (&wd)[4]) {
    const U4 w = philox4x32_10(U4{(uint32_t)j, (uint32_t)quad, (uint32_t)ctr, (uint32_t)(ctr >> 32)}, k0, k1);
    wd[0] = w.x;
    wd[1] = w.y;
    wd[2] = w.z;
    wd[3] = w.w;
}

// Draw-pass state of four rows, updated without branches (a filtered-out element
// arrives as z = key = -inf and changes nothing, except that a chunk with no
// survivor reports its first column with key -inf, which every survivor beats);
// flush() writes the rows' block partials.
struct Draw4 {
    float m[4], s1[4], bk[4];
    int32_t bi[4];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            m[i] = kNegInf;
            s1[i] = 0.f;
            bk[i] = kNegInf;
            bi[i] = 0x7fffffff;
        }
    }
    __device__ __forceinline__ void add(int i, float z, float key, int32_t j) {
        soft_fold1(m[i], s1[i], z);
        const bool win = (key > bk[i]) | ((key == bk[i]) & ((uint32_t)j < (uint32_t)bi[i]));  // no short-circuit branch
        bk[i] = win ? key : bk[i];
        bi[i] = win ? j : bi[i];
    }
    __device__ __forceinline__ void flush(float *red, int64_t b0, int64_t B, int S, int s, Partial *part) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            SoftState st{m[i], s1[i], 0.f};
            block_partial(st, bk[i], bi[i], red);
            if (threadIdx.x == 0 && b0 + i < B) part[(b0 + i) * S + s] = Partial{st.m, st.s1, bk[i], bi[i]};
        }
    }
};

// row_foreach in groups of up to kPerVec<DT> consecutive columns: f(j0, x[PV], n) with
// x[k] the value of column j0 + k for k < n (the rest unset), so a pass can fold a
// whole vector at once (one online-softmax rescale per vector instead of per element).
template <int DT, typename F>
__device__ __forceinline__ void row_foreach_vec(const typename Elem<DT>::T *row, int64_t begin, int64_t end, int tid,
                                                int nthreads, F &&f) {
    using T = typename Elem<DT>::T;
    constexpr int PV = kPerVec<DT>;
    if (end <= begin) return;
    const uintptr_t a = reinterpret_cast<uintptr_t>(row + begin);
    int64_t head = (int64_t)(((16 - (a & 15)) & 15) / sizeof(T));
    if ((a & (sizeof(T) - 1)) != 0) head = end - begin;
    if (head > end - begin) head = end - begin;
    float x[PV];
    for (int64_t j = begin + tid; j < begin + head; j += nthreads) {
        x[0] = Elem<DT>::load(row + j);
        f(j, x, 1);
    }
    const int64_t b0 = begin + head;
    const int64_t nvec = (end - b0) / PV;
    const uint4 *vp = reinterpret_cast<const uint4 *>(row + b0);
    constexpr int U = 4;
    int64_t v = tid;
    for (; v + (U - 1) * (int64_t)nthreads < nvec; v += U * (int64_t)nthreads) {
        uint4 raw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) raw[u] = vp[v + u * nthreads];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            unpack16<DT>(raw[u], x);
            f(b0 + (v + u * nthreads) * PV, x, PV);
        }
    }
    for (; v < nvec; v += nthreads) {
        unpack16<DT>(vp[v], x);
        f(b0 + v * PV, x, PV);
    }
    for (int64_t j = b0 + nvec * PV + tid; j < end; j += nthreads) {
        x[0] = Elem<DT>::load(row + j);
        f(j, x, 1);
    }
}

__device__ __forceinline__ void split_range(int64_t V, int64_t chunk, int64_t &beg, int64_t &end) {
    beg = (int64_t)blockIdx.x * chunk;
    end = beg + chunk < V ? beg + chunk : V;
}

// draw-pass splits per row quad, for about kDrawWgs workgroups
inline int draw_split(int64_t B, int64_t V) {
    const int64_t quads = (B + 3) / 4;
    int S = 1;
    while (S < kMaxDrawSplit && quads * S < kDrawWgs && V / (S * 2) >= 512) S *= 2;
    return S;
}

// ---------------------------------------------------------------------------
// Unfiltered: split rows.
// ---------------------------------------------------------------------------
template <int DT>
__global__ __launch_bounds__(kSplitThreads) void sample_split_kernel(
    const typename Elem<DT>::T *__restrict__ logits, int64_t V, int64_t ld, int64_t B, swh_sample_params p,
    const uint64_t *__restrict__ rng, const int32_t *__restrict__ step_p, const uint32_t *__restrict__ seen,
    int64_t words, int64_t chunk, Partial *__restrict__ part, float *__restrict__ scores_out) {
    __shared__ float red[5 * (kSplitThreads / kWave)];
    const int64_t q = blockIdx.y, b0 = 4 * q;
    const int S = gridDim.x, s = blockIdx.x;
    const int32_t step = *step_p;
    const Proc pr = make_proc(p, step, nullptr);
    const bool pen = p.repetition_penalty != 1.0f && seen;
    float *const srow = scores_out ? scores_out + b0 * V : nullptr;  // rows b0 .. b0 + 3 at V apart
    const uint64_t seed = rng[0], ctr = rng[1] + (uint64_t)step;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    int64_t beg, end;
    split_range(V, chunk, beg, end);
    Draw4 d;
    d.init();
    row4_foreach<DT>(logits, ld, b0, B, beg, end, threadIdx.x, kSplitThreads, [&](int64_t j, const float (&x)[4]) {
        uint32_t wd[4] = {0u, 0u, 0u, 0u};
        if (!p.greedy) philox_col(k0, k1, j, q, ctr, wd);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t b = b0 + i < B ? b0 + i : B - 1;
            const float z = pr.at(j, x[i], pen ? seen + b * words : nullptr);
            if (srow && b0 + i < B) srow[i * V + j] = z;
            d.add(i, z, p.greedy ? z : z + gumbel_from_bits(wd[i]), (int32_t)j);
        }
    });
    d.flush(red, b0, B, S, s, part);
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

constexpr int kFiltSplit = 32;  // workgroups per filtered row (at most)

// Filtered rows over S workgroups each.  Every pass is split like the
// unfiltered path (one workgroup per row ran 64 rows on 64 CUs, and its LDS
// histogram atomics piled onto the few exponent bins most scores share: 549 us
// at 64 x 151936, top-p 0.9).  A threshold is an 11/11/10-bit radix select over
// the order-preserving key of z: each split writes its own 2048-bin partial
// histogram of the next digit, and a per-row select launch sums the S partials
// in fixed order, takes the HIGHEST bin whose inclusive suffix weight reaches
// the target (a max-reduction, robust to float reassociation) and advances the
// row's state in the workspace.  A filter whose total weight stays below its
// target keeps everything.
struct FiltRow {
    float M, lse, lo, above;  // row max, log-normaliser of the weights, threshold, weight above the bin
    uint32_t prefix, pmask;   // key bits resolved so far
    int32_t active, pad;      // 0: the current filter keeps everything
};

struct FiltWs {
    FiltRow *row;  // [B]
    float2 *soft;  // [B][S] (max, sum e^(z - max)) partials
    float *hist;   // [B][S][kBins]
};

inline FiltWs filt_ws(void *ws, int64_t B) {
    char *base = static_cast<char *>(ws) + B * kMaxDrawSplit * (int64_t)sizeof(Partial);
    FiltWs w;
    w.row = reinterpret_cast<FiltRow *>(base);
    base += B * (int64_t)sizeof(FiltRow);
    w.soft = reinterpret_cast<float2 *>(base);
    base += B * kFiltSplit * (int64_t)sizeof(float2);
    w.hist = reinterpret_cast<float *>(base);
    return w;
}

// (max, sum) of the processed scores >= the row threshold (st null: all) over split blockIdx.x
template <int DT>
__global__ __launch_bounds__(kSplitThreads) void filt_soft_kernel(
    const typename Elem<DT>::T *__restrict__ logits, int64_t V, int64_t ld, swh_sample_params p,
    const int32_t *__restrict__ step_p, const uint32_t *__restrict__ seen, int64_t words, int64_t chunk,
    const FiltRow *__restrict__ st, float2 *__restrict__ psoft) {
    __shared__ float red[5 * (kSplitThreads / kWave)];
    const int64_t b = blockIdx.y;
    const Proc pr = make_proc(p, *step_p, seen ? seen + b * words : nullptr);
    const float lo = st ? st[b].lo : kNegInf;
    int64_t beg, end;
    split_range(V, chunk, beg, end);
    SoftState sf = soft_init();
    constexpr int PV = kPerVec<DT>;
    row_foreach_vec<DT>(logits + b * ld, beg, end, threadIdx.x, kSplitThreads,
                        [&](int64_t j0, const float (&x)[PV], int n) {
                            float z[PV];
#pragma unroll
                            for (int k = 0; k < PV; ++k) {
                                const float zk = k < n ? pr(j0 + k, x[k]) : kNegInf;
                                z[k] = zk >= lo ? zk : kNegInf;
                            }
                            soft_fold<PV>(sf, z);  // one rescale per vector
                        });
    sf = block_soft(sf, red);
    if (threadIdx.x == 0) psoft[b * gridDim.x + blockIdx.x] = float2{sf.m, sf.s1};
}

// Opens a filter: mode 0 also records the row max and sets the threshold to -inf
// (the log-normaliser of all scores); mode 1 takes the log-normaliser of the
// survivors of the previous filter.
__global__ __launch_bounds__(64) void filt_row_kernel(FiltRow *__restrict__ st, const float2 *__restrict__ psoft,
                                                      int S, int mode) {
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    SoftState a = soft_init();
    for (int q = lane; q < S; q += 64) a = soft_merge(a, SoftState{psoft[b * S + q].x, psoft[b * S + q].y, 0.f});
    a = wave_soft(a);
    if (lane != 0) return;
    FiltRow r = st[b];
    if (mode == 0) {
        r.M = a.m;
        r.lo = kNegInf;
    }
    r.lse = a.m + fast_log(a.s1);
    r.above = 0.f;
    r.prefix = 0u;
    r.pmask = 0u;
    r.active = 1;
    st[b] = r;
}

// Partial histogram of digit `lvl` over split blockIdx.x: scores >= lo whose
// resolved key bits match, weighted 1 (top-k) or e^(z - lse) (top-p).  Runs of
// equal bins within a thread's elements are summed in registers first (scores
// mostly share a few exponent bins), one LDS atomic per run.  The weights are
// summed as 2^-40 fixed point in 64-bit integers: integer adds commute, so the
// bins (and the threshold) are the same in every run — float LDS atomics made
// the top-p draw run-to-run nondeterministic (their order varies).  Sums stay
// below V 2^40 < 2^64; a weight under 2^-40 (probability < e^-27.7) adds 0.
constexpr float kHistScale = 1099511627776.0f;  // 2^40
template <int DT, bool EXPW>
__global__ __launch_bounds__(kSplitThreads) void filt_hist_kernel(
    const typename Elem<DT>::T *__restrict__ logits, int64_t V, int64_t ld, swh_sample_params p,
    const int32_t *__restrict__ step_p, const uint32_t *__restrict__ seen, int64_t words, int64_t chunk,
    const FiltRow *__restrict__ st, int lvl, float *__restrict__ phist) {
    __shared__ unsigned long long hist[kBins];
    const int64_t b = blockIdx.y;
    const int t = threadIdx.x;
    const FiltRow r = st[b];
    if (!r.active) return;
    const int sh = lvl == 0 ? 21 : (lvl == 1 ? 10 : 0);
    const uint32_t dmask = lvl == 2 ? 0x3ffu : 0x7ffu;
    for (int i = t; i < kBins; i += kSplitThreads) hist[i] = 0ull;
    __syncthreads();
    const Proc pr = make_proc(p, *step_p, seen ? seen + b * words : nullptr);
    int64_t beg, end;
    split_range(V, chunk, beg, end);
    int run_bin = -1;
    unsigned long long run_w = 0ull;
    row_foreach<DT, false>(logits + b * ld, beg, end, t, kSplitThreads, [&](int64_t j, float x) {
        const float z = pr(j, x);
        if (!(z >= r.lo) || z == kNegInf) return;
        const uint32_t k = ord_key(z);
        if ((k & r.pmask) != r.prefix) return;
        const int bin = (int)((k >> sh) & dmask);
        const unsigned long long w = (unsigned long long)((EXPW ? fast_exp(z - r.lse) : 1.0f) * kHistScale);
        if (bin == run_bin) {
            run_w += w;
        } else {
            if (run_bin >= 0) atomicAdd(&hist[run_bin], run_w);
            run_bin = bin;
            run_w = w;
        }
    });
    if (run_bin >= 0) atomicAdd(&hist[run_bin], run_w);
    __syncthreads();
    float *dst = phist + (b * gridDim.x + blockIdx.x) * (int64_t)kBins;
    for (int i = t; i < kBins; i += kSplitThreads) dst[i] = (float)((double)hist[i] * (1.0 / 1099511627776.0));
}

// One radix level per row: the bin of digit `lvl` where the weight from the top
// reaches `target`; the last level turns the resolved key into the threshold.
__global__ __launch_bounds__(kFiltThreads) void filt_select_kernel(FiltRow *__restrict__ st,
                                                                    const float *__restrict__ phist, int S, int lvl,
                                                                    float target) {
    __shared__ float scan[64];
    __shared__ int sel[2];
    const int64_t b = blockIdx.x;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6, nw = kFiltThreads >> 6;
    const FiltRow r = st[b];
    if (!r.active) return;
    const int sh = lvl == 0 ? 21 : (lvl == 1 ? 10 : 0);
    const uint32_t dmask = lvl == 2 ? 0x3ffu : 0x7ffu;
    float h0 = 0.f, h1 = 0.f;
    for (int q = 0; q < S; ++q) {  // splits in fixed order
        const float *h = phist + (b * S + q) * (int64_t)kBins;
        h0 += h[2 * t];
        h1 += h[2 * t + 1];
    }
    if (t == 0) {
        sel[0] = -1;
        sel[1] = kBins;
    }
    __syncthreads();
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
    const float a1 = r.above + (v - tsum) + after;  // weight strictly above bin 2t+1
    const float a0 = a1 + h1;                       // weight strictly above bin 2t
    int cand = -1;
    if (h1 > 0.f && a1 + h1 >= target) cand = 2 * t + 1;
    else if (h0 > 0.f && a0 + h0 >= target) cand = 2 * t;
    if (cand >= 0) atomicMax(&sel[0], cand);
    if (h0 > 0.f) atomicMin(&sel[1], 2 * t);
    else if (h1 > 0.f) atomicMin(&sel[1], 2 * t + 1);
    __syncthreads();
    int bin = sel[0];
    if (bin < 0) {
        if (lvl == 0) {  // the filter's total weight stays below its target: keep everything
            if (t == 0) st[b].active = 0;
            return;
        }
        bin = sel[1] < kBins ? sel[1] : 0;
    }
    if (bin == 2 * t + 1) scan[nw] = a1;
    if (bin == 2 * t) scan[nw] = a0;
    __syncthreads();
    if (t == 0) {
        FiltRow w = r;
        w.above = scan[nw];
        w.prefix |= (uint32_t)bin << sh;
        w.pmask |= dmask << sh;
        if (lvl == 2) w.lo = fmaxf(w.lo, key_to_float(w.prefix));
        st[b] = w;
    }
}

// Final pass over split blockIdx.x of a row quad: min-p, then the Gumbel-max draw among the survivors
template <int DT>
__global__ __launch_bounds__(kSplitThreads) void filt_draw_kernel(
    const typename Elem<DT>::T *__restrict__ logits, int64_t V, int64_t ld, int64_t B, swh_sample_params p,
    const uint64_t *__restrict__ rng, const int32_t *__restrict__ step_p, const uint32_t *__restrict__ seen,
    int64_t words, int64_t chunk, const FiltRow *__restrict__ st, Partial *__restrict__ part,
    float *__restrict__ scores_out) {
    __shared__ float red[5 * (kSplitThreads / kWave)];
    const int64_t q = blockIdx.y, b0 = 4 * q;
    const int32_t step = *step_p;
    const Proc pr = make_proc(p, step, nullptr);
    const bool pen = p.repetition_penalty != 1.0f && seen;
    float lo[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const FiltRow r = st[b0 + i < B ? b0 + i : B - 1];
        lo[i] = r.lo;
        // min-p: p_j < min_p * p_max  <=>  z_j < M + ln(min_p)
        if (p.min_p > 0.f) lo[i] = fmaxf(lo[i], r.M + logf(p.min_p));
    }
    float *const srow = scores_out ? scores_out + b0 * V : nullptr;
    const uint64_t seed = rng[0], ctr = rng[1] + (uint64_t)step;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    int64_t beg, end;
    split_range(V, chunk, beg, end);
    Draw4 d;
    d.init();
    row4_foreach<DT>(logits, ld, b0, B, beg, end, threadIdx.x, kSplitThreads, [&](int64_t j, const float (&x)[4]) {
        uint32_t wd[4];
        philox_col(k0, k1, j, q, ctr, wd);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t b = b0 + i < B ? b0 + i : B - 1;
            float z = pr.at(j, x[i], pen ? seen + b * words : nullptr);
            if (!(z >= lo[i])) z = kNegInf;
            if (srow && b0 + i < B) srow[i * V + j] = z;
            d.add(i, z, z + gumbel_from_bits(wd[i]), (int32_t)j);
        }
    });
    d.flush(red, b0, B, gridDim.x, blockIdx.x, part);
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

// ---------------------------------------------------------------------------
// Filtered, bf16 logits without a repetition penalty: one top-k or one top-p
// threshold (min-p as in the general path).  Processing (EOS suppression, / T)
// is monotone in the bf16 logit, so the threshold is a 16-bit radix select over
// the order-preserving key of the bf16 BITS (two 8-bit digits, 256 bins) instead
// of three digits over the fp32 score, and the per-row select runs in the
// prologue of the pass that needs it — every split workgroup of a row sums the
// row's S partial histograms in the same fixed order, so all agree — instead of
// in separate launches: soft, digit 0, digit 1, draw (4 launches + the finalize,
// against 10).  The kept set, ties at the threshold included, and the draws are
// those of the general path.
// ---------------------------------------------------------------------------
constexpr int kBins16 = 256;

__device__ __forceinline__ uint32_t ord_key16(float x) {  // x holds a bf16 value exactly
    const uint32_t u = __float_as_uint(x) >> 16;
    return (u & 0x8000u) ? (~u & 0xffffu) : (u | 0x8000u);
}

struct Filt16Row {
    float M, lse;     // row max and log-normaliser of the processed scores
    float above;      // weight strictly above the selected digit-0 bin
    int32_t thr;      // the resolved key prefix (digit 0: bin << 8; final: the 16-bit threshold key)
    int32_t active;   // 0: the filter keeps everything
};

// The row's (max, lse) from the S soft partials (fixed order).
__device__ __forceinline__ void row_soft16(const float2 *__restrict__ psoft, int64_t b, int S, float &M, float &lse) {
    if (!psoft) {  // a top-k without min-p weighs nothing by the scores: no soft pass ran
        M = lse = 0.f;
        return;
    }
    SoftState a = soft_init();
    for (int q = 0; q < S; ++q) a = soft_merge(a, SoftState{psoft[b * S + q].x, psoft[b * S + q].y, 0.f});
    M = a.m;
    lse = a.m + fast_log(a.s1);
}

// Select over the S partial 256-bin histograms of row b (kSplitThreads == 256 threads,
// thread t owns bin t): the highest bin whose weight from the top reaches `target`
// given `above0` above all bins.  Returns the bin (-1: total below target) and the
// weight strictly above it; `lowest`: the lowest non-empty bin (the level-1 fallback).
__device__ __forceinline__ int select16(const float *__restrict__ phist, int64_t b, int S, float above0, float target,
                                        float &above, int &lowest, float *scan, int *sel,
                                        const float *fs = nullptr) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6, nw = kSplitThreads >> 6;
    float h = 0.f;
    for (int q = 0; q < S; ++q) {  // splits in fixed order; fs: each split's weight scale (LDS)
        const float v = phist[(b * S + q) * (int64_t)kBins16 + t];
        h += fs ? v * fs[q] : v;
    }
    if (t == 0) {
        sel[0] = -1;
        sel[1] = kBins16;
    }
    float v = h;  // inclusive suffix scan over lanes (higher lanes = higher bins)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const float u = __shfl_down(v, o, kWave);
        if (lane + o < 64) v += u;
    }
    if (lane == 0) scan[wid] = v;  // the wave's total
    __syncthreads();
    float after = 0.f;
    for (int w = wid + 1; w < nw; ++w) after += scan[w];
    const float a = above0 + (v - h) + after;  // weight strictly above bin t
    if (h > 0.f && a + h >= target) atomicMax(&sel[0], t);
    if (h > 0.f) atomicMin(&sel[1], t);
    __syncthreads();
    const int bin = sel[0];
    if (bin == t) scan[nw] = a;
    const int lo = sel[1];
    if (bin < 0 && lo == t) scan[nw] = a;
    __syncthreads();
    above = scan[nw];
    lowest = lo;
    const int r = bin;
    __syncthreads();  // scan / sel are reused by the caller
    return r;
}

// Digit LVL's partial histogram over split blockIdx.x.  LVL 0: weights e^(z - lse)
// (top-p) or 1 (top-k) of the processed scores, binned by the top byte of the key;
// LVL 1: the prologue resolves digit 0 (and writes the row state once), then bins
// the low byte of the keys under that prefix.
template <bool EXPW, int LVL>
__global__ __launch_bounds__(kSplitThreads) void filt16_hist_kernel(
    const uint16_t *__restrict__ logits, int64_t V, int64_t ld, swh_sample_params p, const int32_t *__restrict__ step_p,
    int64_t chunk, const float2 *__restrict__ psoft, const float *__restrict__ phist0, float target,
    Filt16Row *__restrict__ rows, float *__restrict__ phist) {
    __shared__ unsigned long long hist[kBins16];
    __shared__ float scan[kSplitThreads / kWave + 1];
    __shared__ int sel[2];
    const int64_t b = blockIdx.y;
    const int t = threadIdx.x, S = gridDim.x;
    float M, lse;
    row_soft16(psoft, b, S, M, lse);
    int prefix = 0;
    if constexpr (LVL == 1) {
        // top-p: the digit-0 partials weigh e^(z - m_s) by their own split max (filt16_soft_hist0_kernel);
        // e^(m_s - lse) puts them on the row's scale
        __shared__ float fs[kFiltSplit];
        if (EXPW && t < S) fs[t] = fast_exp(psoft[b * S + t].x - lse);
        __syncthreads();
        float above;
        int lowest;
        const int bin = select16(phist0, b, S, 0.f, target, above, lowest, scan, sel, EXPW ? fs : nullptr);
        if (bin < 0) {  // the filter's total weight stays below its target: keep everything
            if (blockIdx.x == 0 && t == 0) rows[b] = Filt16Row{M, lse, 0.f, 0, 0};
            return;
        }
        prefix = bin;
        if (blockIdx.x == 0 && t == 0) rows[b] = Filt16Row{M, lse, above, bin << 8, 1};
    }
    hist[t] = 0ull;
    __syncthreads();
    const Proc pr = make_proc(p, *step_p, nullptr);
    int64_t beg, end;
    split_range(V, chunk, beg, end);
    int run_bin = -1;
    unsigned long long run_w = 0ull;
    row_foreach<SWH_BF16, false>(logits + b * ld, beg, end, t, kSplitThreads, [&](int64_t j, float x) {
        const float z = pr(j, x);
        if (z == kNegInf) return;
        const uint32_t k = ord_key16(x);
        if (LVL == 1 && (int)(k >> 8) != prefix) return;
        const int bin = LVL == 0 ? (int)(k >> 8) : (int)(k & 0xffu);
        const unsigned long long w = (unsigned long long)((EXPW ? fast_exp(z - lse) : 1.0f) * kHistScale);
        if (bin == run_bin) {
            run_w += w;
        } else {
            if (run_bin >= 0) atomicAdd(&hist[run_bin], run_w);
            run_bin = bin;
            run_w = w;
        }
    });
    if (run_bin >= 0) atomicAdd(&hist[run_bin], run_w);
    __syncthreads();
    phist[(b * S + blockIdx.x) * (int64_t)kBins16 + t] = (float)((double)hist[t] * (1.0 / 1099511627776.0));
}

// Top-p, split blockIdx.x: the soft partial (split max m_s, sum e^(z - m_s)) and the
// digit-0 histogram in ONE launch — the split's max first (a read of its chunk), then
// the histogram weighs e^(z - m_s) (2^-40 fixed point, as filt16_hist_kernel) while the
// sum accumulates; the digit-1 pass rescales each split's bins by e^(m_s - lse).  The
// second read of the chunk comes from the caches.
__global__ __launch_bounds__(kSplitThreads) void filt16_soft_hist0_kernel(
    const uint16_t *__restrict__ logits, int64_t V, int64_t ld, swh_sample_params p, const int32_t *__restrict__ step_p,
    int64_t chunk, float2 *__restrict__ psoft, float *__restrict__ phist) {
    __shared__ unsigned long long hist[kBins16];
    __shared__ float red[5 * (kSplitThreads / kWave)];
    const int64_t b = blockIdx.y;
    const int t = threadIdx.x, S = gridDim.x;
    const Proc pr = make_proc(p, *step_p, nullptr);
    int64_t beg, end;
    split_range(V, chunk, beg, end);
    const uint16_t *row = logits + b * ld;
    float m = kNegInf;
    row_foreach_vec<SWH_BF16>(row, beg, end, t, kSplitThreads, [&](int64_t j0, const float (&x)[8], int n) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (k < n) m = fmaxf(m, pr(j0 + k, x[k]));
    });
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, kWave));
    if ((t & 63) == 0) red[t >> 6] = m;
    hist[t] = 0ull;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    static_assert(kSplitThreads == 4 * kWave, "four waves");
    __syncthreads();  // red is reused by block_soft
    float sum = 0.f;
    int run_bin = -1;
    unsigned long long run_w = 0ull;
    if (m != kNegInf) {
        row_foreach<SWH_BF16, false>(row, beg, end, t, kSplitThreads, [&](int64_t j, float x) {
            const float z = pr(j, x);
            if (z == kNegInf) return;
            const float e = fast_exp(z - m);
            sum += e;
            const int bin = (int)(ord_key16(x) >> 8);
            const unsigned long long w = (unsigned long long)(e * kHistScale);
            if (bin == run_bin) {
                run_w += w;
            } else {
                if (run_bin >= 0) atomicAdd(&hist[run_bin], run_w);
                run_bin = bin;
                run_w = w;
            }
        });
    }
    if (run_bin >= 0) atomicAdd(&hist[run_bin], run_w);
    const SoftState st = block_soft(SoftState{m, sum, 0.f}, red);  // equal maxima: the sums add
    if (t == 0) psoft[b * S + blockIdx.x] = float2{st.m, st.s1};
    phist[(b * S + blockIdx.x) * (int64_t)kBins16 + t] = (float)((double)hist[t] * (1.0 / 1099511627776.0));
}

// Final pass over split blockIdx.x: the prologue resolves digit 1 (the 16-bit
// threshold key), then min-p and the Gumbel-max draw among the survivors, with the
// survivors' (max, sum) for the finalize's log-prob.
__global__ __launch_bounds__(kSplitThreads) void filt16_draw_kernel(
    const uint16_t *__restrict__ logits, int64_t V, int64_t ld, swh_sample_params p, const uint64_t *__restrict__ rng,
    const int32_t *__restrict__ step_p, int64_t chunk, const float2 *__restrict__ psoft, const float *__restrict__ phist1,
    float target, int filtered, const Filt16Row *__restrict__ rows, Partial *__restrict__ part,
    float *__restrict__ scores_out) {
    __shared__ float red[5 * (kSplitThreads / kWave)];
    __shared__ float scan[kSplitThreads / kWave + 1];
    __shared__ int sel[2];
    const int64_t b = blockIdx.y;
    const int S = gridDim.x;
    float M, lse;
    row_soft16(psoft, b, S, M, lse);
    int thr = -1;  // keys >= thr survive (-1: all)
    if (filtered) {
        const Filt16Row r = rows[b];
        if (r.active) {
            float above;
            int lowest;
            int bin = select16(phist1, b, S, r.above, target, above, lowest, scan, sel);
            if (bin < 0) bin = lowest < kBins16 ? lowest : 0;
            thr = r.thr | bin;
        }
    }
    float lo = kNegInf;
    if (p.min_p > 0.f) lo = M + logf(p.min_p);  // p_j < min_p * p_max  <=>  z_j < M + ln(min_p)
    const int32_t step = *step_p;
    const Proc pr = make_proc(p, step, nullptr);
    const uint64_t seed = rng[0], ctr = rng[1] + (uint64_t)step;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    int64_t beg, end;
    split_range(V, chunk, beg, end);
    SoftState sf = soft_init();
    float bk = kNegInf;
    int32_t bi = 0x7fffffff;
    float *srow = scores_out ? scores_out + b * V : nullptr;
    row_foreach_vec<SWH_BF16>(logits + b * ld, beg, end, threadIdx.x, kSplitThreads,
                              [&](int64_t j0, const float (&x)[8], int n) {
                                  float z[8];
#pragma unroll
                                  for (int k = 0; k < 8; ++k) {
                                      const float zk = k < n ? pr(j0 + k, x[k]) : kNegInf;
                                      z[k] = ((int)ord_key16(x[k]) < thr || !(zk >= lo)) ? kNegInf : zk;
                                      if (srow && k < n) srow[j0 + k] = z[k];
                                  }
                                  soft_fold<8>(sf, z);  // one rescale per vector
#pragma unroll
                                  for (int k = 0; k < 8; ++k)
                                      if (z[k] != kNegInf)
                                          best_merge(bk, bi, z[k] + gumbel_at(k0, k1, j0 + k, b, ctr), (int32_t)(j0 + k));
                              });
    block_partial(sf, bk, bi, red);
    if (threadIdx.x == 0) part[b * S + blockIdx.x] = Partial{sf.m, sf.s1, bk, bi};
}

// true when the 16-bit path serves these parameters (one threshold, no penalty, bf16)
inline bool filt16_serves(const swh_sample_params &p, int64_t V) {
    const bool topk = p.top_k > 0 && p.top_k < V, topp = p.top_p < 1.0f;
    return p.repetition_penalty == 1.0f && !(topk && topp);
}

int launch_filtered16(const uint16_t *lg, int64_t B, int64_t V, int64_t ld, const swh_sample_params &p,
                      const uint64_t *rng, const int32_t *step, void *workspace, float *scores_out, hipStream_t s) {
    const int target_wgs = launch_policy().filt_wgs;
    int S = 1;
    while (S < kFiltSplit && B * S < target_wgs && V / (S * 2) >= 2048) S *= 2;
    int64_t chunk = (V + S - 1) / S;
    chunk = (chunk + 7) / 8 * 8;
    const FiltWs w = filt_ws(workspace, B);
    Partial *part = static_cast<Partial *>(workspace);
    auto *rows = reinterpret_cast<Filt16Row *>(w.row);  // sizeof(Filt16Row) <= sizeof(FiltRow)
    float *h0 = w.hist, *h1 = w.hist + B * kFiltSplit * (int64_t)kBins16;
    const dim3 gs((unsigned)S, (unsigned)B);
    const bool topk = p.top_k > 0 && p.top_k < V, topp = p.top_p < 1.0f;
    const bool filtered = topk || topp;
    const float target = topk ? (float)p.top_k : p.top_p;
    // the row max / log-normaliser: top-p weights and min-p need them; a count threshold does not
    const float2 *soft = (topp || p.min_p > 0.f) ? w.soft : nullptr;
    if (soft && !topp) filt_soft_kernel<SWH_BF16><<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, step, nullptr, 0, chunk,
                                                                               nullptr, w.soft);
    if (filtered) {
        if (topk) {
            filt16_hist_kernel<false, 0><<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, step, chunk, soft, nullptr, target,
                                                                      rows, h0);
            filt16_hist_kernel<false, 1><<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, step, chunk, soft, h0, target,
                                                                      rows, h1);
        } else {
            filt16_soft_hist0_kernel<<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, step, chunk, w.soft, h0);
            filt16_hist_kernel<true, 1><<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, step, chunk, w.soft, h0, target,
                                                                     rows, h1);
        }
    }
    filt16_draw_kernel<<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, rng, step, chunk, soft, h1, target,
                                                    filtered ? 1 : 0, rows, part, scores_out);
    return S;
}

template <int DT>
int launch_filtered(const typename Elem<DT>::T *lg, int64_t B, int64_t V, int64_t ld, const swh_sample_params &p,
                    const uint64_t *rng, const int32_t *step, const uint32_t *seen, int64_t words, void *workspace,
                    float *scores_out, hipStream_t s) {
    // more splits than the unfiltered path: each digit pass is bound by its
    // workgroups' LDS histogram atomics, so spread a row over up to the policy's filt_wgs
    const int target = launch_policy().filt_wgs;
    int S = 1;
    while (S < kFiltSplit && B * S < target && V / (S * 2) >= 2048) S *= 2;
    int64_t chunk = (V + S - 1) / S;
    chunk = (chunk + 7) / 8 * 8;
    const FiltWs w = filt_ws(workspace, B);
    Partial *part = static_cast<Partial *>(workspace);
    const dim3 gs((unsigned)S, (unsigned)B), gr((unsigned)B);
    filt_soft_kernel<DT><<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, step, seen, words, chunk, nullptr, w.soft);
    filt_row_kernel<<<gr, 64, 0, s>>>(w.row, w.soft, S, 0);
    const bool topk = p.top_k > 0 && p.top_k < V;
    if (topk) {  // count threshold
        for (int lvl = 0; lvl < 3; ++lvl) {
            filt_hist_kernel<DT, false><<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, step, seen, words, chunk, w.row,
                                                                     lvl, w.hist);
            filt_select_kernel<<<gr, kFiltThreads, 0, s>>>(w.row, w.hist, S, lvl, (float)p.top_k);
        }
    }
    if (p.top_p < 1.0f) {  // mass threshold, renormalised over the top-k survivors
        if (topk) {
            filt_soft_kernel<DT><<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, step, seen, words, chunk, w.row, w.soft);
            filt_row_kernel<<<gr, 64, 0, s>>>(w.row, w.soft, S, 1);
        }
        for (int lvl = 0; lvl < 3; ++lvl) {
            filt_hist_kernel<DT, true><<<gs, kSplitThreads, 0, s>>>(lg, V, ld, p, step, seen, words, chunk, w.row,
                                                                    lvl, w.hist);
            filt_select_kernel<<<gr, kFiltThreads, 0, s>>>(w.row, w.hist, S, lvl, p.top_p);
        }
    }
    const int Sd = draw_split(B, V);
    int64_t cd = (V + Sd - 1) / Sd;
    cd = (cd + 7) / 8 * 8;
    filt_draw_kernel<DT><<<dim3((unsigned)Sd, (unsigned)((B + 3) / 4)), kSplitThreads, 0, s>>>(
        lg, V, ld, B, p, rng, step, seen, words, cd, w.row, part, scores_out);
    return Sd;
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int64_t swh_sample_workspace_bytes(int64_t B, int64_t V) {
    (void)V;  // [split partials | filtered rows: state, (max, sum) partials, digit histograms]
    return B * kMaxDrawSplit * (int64_t)sizeof(Partial) + B * (int64_t)sizeof(FiltRow) +
           B * kFiltSplit * (int64_t)sizeof(float2) + B * kFiltSplit * kBins * (int64_t)sizeof(float);
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
        if (filtered && DTC == SWH_BF16 && filt16_serves(p, V)) {                                              \
            S = launch_filtered16(reinterpret_cast<const uint16_t *>(lg), B, V, ld, p, rng, step, workspace,    \
                                  scores_out, s);                                                               \
        } else if (filtered) {                                                                                  \
            S = launch_filtered<DTC>(lg, B, V, ld, p, rng, step, seen, words, workspace, scores_out, s);         \
        } else {                                                                                                \
            S = draw_split(B, V);                                                                               \
            int64_t chunk = (V + S - 1) / S;                                                                    \
            chunk = (chunk + 7) / 8 * 8;                                                                        \
            sample_split_kernel<DTC><<<dim3((unsigned)S, (unsigned)((B + 3) / 4)), dim3(kSplitThreads), 0, s>>>( \
                lg, V, ld, B, p, rng, step, seen, words, chunk, part, scores_out);                              \
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
