// GRPO / PPO per-token math on device: completion mask, group advantages,
// the fused GRPO loss forward+backward, masked whitening, GAE, PPO losses and
// the value head.  All are tiny next to the logits-sized kernels; they exist so
// the step has no host round-trip and no chain of ~20 elementwise launches.
//
// Reductions are deterministic: one workgroup, fixed per-thread order, wave
// shuffles, then a fixed-order LDS merge.
#include "common.hpp"

namespace swh {
namespace {

constexpr int kBig = 1024;

// ---------------------------------------------------------------------------
// a5 — grpo_trainer.py:1812-1831
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void completion_mask_kernel(const int64_t *__restrict__ ids, int64_t C,
                                                              const int32_t *__restrict__ eos, int32_t n_eos,
                                                              int32_t mask_trunc, int32_t *__restrict__ mask,
                                                              int32_t *__restrict__ lengths,
                                                              int32_t *__restrict__ has_eos) {
    __shared__ int32_t first;
    const int64_t b = blockIdx.x;
    if (threadIdx.x == 0) first = (int32_t)C;
    __syncthreads();
    int32_t mine = (int32_t)C;
    for (int64_t t = threadIdx.x; t < C; t += blockDim.x) {
        const int64_t v = ids[b * C + t];
        bool e = false;
        for (int k = 0; k < n_eos; ++k) e |= (v == eos[k]);
        if (e) {
            mine = (int32_t)t;
            break;
        }
    }
    atomicMin(&first, mine);
    __syncthreads();
    const int32_t f = first;
    const bool has = f < C;
    const int32_t keep = (mask_trunc && !has) ? 0 : 1;
    for (int64_t t = threadIdx.x; t < C; t += blockDim.x) mask[b * C + t] = (t <= f) ? keep : 0;
    if (threadIdx.x == 0) {
        if (lengths) lengths[b] = has ? f + 1 : (int32_t)C;  // before truncation masking (:1826)
        if (has_eos) has_eos[b] = has ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// a10 — grpo_trainer.py:1914-1930 (one thread per group)
// ---------------------------------------------------------------------------
__global__ void group_advantage_kernel(const float *__restrict__ rpf, const float *__restrict__ w, int64_t N,
                                       int64_t F, int64_t G, int32_t scale, float *__restrict__ adv,
                                       float *__restrict__ rew, float *__restrict__ gmean,
                                       float *__restrict__ gstd, int32_t *__restrict__ zstd) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g * G >= N) return;
    double sum = 0.0;
    for (int64_t i = 0; i < G; ++i) {
        float r = 0.f;
        for (int64_t f = 0; f < F; ++f) {
            const float x = rpf[(g * G + i) * F + f] * w[f];
            if (!__builtin_isnan(x)) r += x;  // nansum
        }
        if (rew) rew[g * G + i] = r;
        sum += r;
    }
    const float mean = (float)(sum / (double)G);
    double ss = 0.0;
    for (int64_t i = 0; i < G; ++i) {
        float r = 0.f;
        for (int64_t f = 0; f < F; ++f) {
            const float x = rpf[(g * G + i) * F + f] * w[f];
            if (!__builtin_isnan(x)) r += x;
        }
        const double d = (double)r - (double)mean;
        ss += d * d;
    }
    const float std = (float)sqrt(ss / (double)(G - 1));  // unbiased (torch.std default)
    for (int64_t i = 0; i < G; ++i) {
        float r = 0.f;
        for (int64_t f = 0; f < F; ++f) {
            const float x = rpf[(g * G + i) * F + f] * w[f];
            if (!__builtin_isnan(x)) r += x;
        }
        float a = r - mean;
        if (scale) a = a / (std + 1e-4f);
        adv[g * G + i] = a;
    }
    if (gmean) gmean[g] = mean;
    if (gstd) gstd[g] = std;
    if (zstd) zstd[g] = (fabsf(std) <= 1e-8f) ? 1 : 0;  // torch.isclose(std, 0)
}

// ---------------------------------------------------------------------------
// a11 — grpo_trainer.py:2058-2175, fused forward + d loss / d logp.
// ---------------------------------------------------------------------------
struct ClipOut {
    float ptl_policy;  // -min(c1' A, c2 A)
    float dpol;        // d(-min)/d x   (x = log importance weight)
    float c1d;         // coef_1 after the delta clamp (metrics)
};

__device__ __forceinline__ ClipOut clip_term(float x, float A, float el, float eh, float delta) {
    const float c1 = expf(x);
    const float c2 = fminf(fmaxf(c1, 1.f - el), 1.f + eh);
    const bool use_delta = delta > 0.f;
    const float c1d = use_delta ? fminf(c1, delta) : c1;
    const float l1 = c1d * A, l2 = c2 * A;
    float g1, g2;
    if (l1 < l2) { g1 = 1.f; g2 = 0.f; }
    else if (l2 < l1) { g1 = 0.f; g2 = 1.f; }
    else { g1 = 0.5f; g2 = 0.5f; }  // torch.min tie: gradient split evenly
    const float dl1 = A * c1 * ((!use_delta || c1 <= delta) ? 1.f : 0.f);
    const float dl2 = A * c1 * ((c1 >= 1.f - el && c1 <= 1.f + eh) ? 1.f : 0.f);
    return ClipOut{-fminf(l1, l2), -(g1 * dl1 + g2 * dl2), c1d};
}

struct LossWS {
    float *row_len;   // [R] sum mask
    float *row_x;     // [R] sequence-level log weight
    float *row_w;     // [R] per-row aggregation factor (w_bt = row_w[b] * m_bt)
    float *row_gx;    // [R] dL/dx_b for sequence level
    float *seg_tok;   // [S]
    float *seg_rows;  // [S]
};

__global__ __launch_bounds__(kBig) void grpo_loss_kernel(
    const float *__restrict__ lp, const float *__restrict__ old, const float *__restrict__ ref,
    const float *__restrict__ adv, const int32_t *__restrict__ mask, const uint8_t *__restrict__ em,
    const float *__restrict__ ent, const float *__restrict__ row_scale, const int32_t *__restrict__ seg,
    int64_t R, int64_t T, swh_grpo_loss_params p, float *__restrict__ loss, float *__restrict__ dlp,
    float *__restrict__ metrics, float *__restrict__ seg_metrics, LossWS ws) {
    __shared__ float red[8 * (kBig / kWave)];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
    const int S = p.num_segments;
    const bool seq = p.is_level == SWH_IS_SEQUENCE;

    // Phase 1: per-row mask length and sequence-level log weight (one wave per row).
    for (int64_t r = wid; r < R; r += nw) {
        float len = 0.f, xs = 0.f;
        for (int64_t t = lane; t < T; t += 64) {
            const float m = (float)mask[r * T + t];
            len += m;
            if (seq) {
                const float d = old ? lp[r * T + t] - old[r * T + t] : 0.f;
                xs += d * m;
            }
        }
        len = wave_sum(len);
        xs = wave_sum(xs);
        if (lane == 0) {
            ws.row_len[r] = len;
            ws.row_x[r] = xs / fmaxf(len, 1.f);
        }
    }
    __syncthreads();
    // Phase 2: per-segment token and row counts (one thread per segment).
    for (int s = tid; s < S; s += blockDim.x) {
        float tok = 0.f, rows = 0.f;
        for (int64_t r = 0; r < R; ++r) {
            const int sr = seg ? seg[r] : 0;
            if (sr == s) {
                tok += ws.row_len[r];
                rows += 1.f;
            }
        }
        ws.seg_tok[s] = tok;
        ws.seg_rows[s] = rows;
    }
    __syncthreads();
    // Phase 3: per-row aggregation factor.
    for (int64_t r = tid; r < R; r += blockDim.x) {
        const int s = seg ? seg[r] : 0;
        const float sc = row_scale ? row_scale[r] : 1.f;
        float f;
        if (p.loss_type == SWH_LOSS_GRPO) f = 1.f / (fmaxf(ws.row_len[r], 1.f) * ws.seg_rows[s]);
        else if (p.loss_type == SWH_LOSS_BNPO) f = 1.f / fmaxf(ws.seg_tok[s], 1.f);
        else f = 1.f / (ws.seg_rows[s] * (float)p.max_completion_length);
        ws.row_w[r] = f * sc;
    }
    __syncthreads();
    // Phase 4 (sequence level): dL/dx_b = row_w * sum_t m*em * d(-min)/dx.
    if (seq) {
        for (int64_t r = wid; r < R; r += nw) {
            const float A = adv[r];
            const ClipOut c = clip_term(ws.row_x[r], A, p.epsilon_low, p.epsilon_high, p.delta);
            float sem = 0.f;
            for (int64_t t = lane; t < T; t += 64) {
                const float m = (float)mask[r * T + t];
                sem += m * (em ? (float)em[r * T + t] : 1.f);
            }
            sem = wave_sum(sem);
            if (lane == 0) ws.row_gx[r] = ws.row_w[r] * sem * c.dpol;
        }
        __syncthreads();
    }
    // Phase 5: elementwise loss, gradient and metric sums.
    float acc[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // loss, tok, kl, ent, low, high, region
    const int64_t N = R * T;
    for (int64_t i = tid; i < N; i += blockDim.x) {
        const int64_t r = i / T;
        const float m = (float)mask[i];
        const float A = adv[r];
        const float l = lp[i];
        const float x = seq ? ws.row_x[r] : (old ? l - old[i] : 0.f);
        const ClipOut c = clip_term(x, A, p.epsilon_low, p.epsilon_high, p.delta);
        const float e = em ? (float)em[i] : 1.f;
        float ptl = c.ptl_policy * e, g = 0.f;
        float kl = 0.f;
        if (p.beta != 0.f) {
            const float d = ref[i] - l;
            const float ed = expf(d);
            kl = ed - d - 1.f;
            ptl += p.beta * kl;
            g += p.beta * (1.f - ed);
        }
        const float w = ws.row_w[r] * m;
        acc[0] += w * ptl;
        if (dlp) {
            float grad = w * g;
            if (seq) grad += ws.row_gx[r] * m / fmaxf(ws.row_len[r], 1.f);
            else grad += w * c.dpol * e;
            dlp[i] = grad;
        }
        acc[1] += m;
        acc[2] += kl * m;
        if (ent) acc[3] += ent[i] * m;
        if (!seq) {
            const float lo = (c.c1d < 1.f - p.epsilon_low && A < 0.f) ? 1.f : 0.f;
            const float hi = (c.c1d > 1.f + p.epsilon_high && A > 0.f) ? 1.f : 0.f;
            acc[4] += lo * m;
            acc[5] += hi * m;
            acc[6] += fmaxf(lo, hi) * m;
        }
    }
    if (seq) {  // clip metrics live on [R, 1]: plain row sums
        for (int64_t r = tid; r < R; r += blockDim.x) {
            const float A = adv[r];
            const ClipOut c = clip_term(ws.row_x[r], A, p.epsilon_low, p.epsilon_high, p.delta);
            const float lo = (c.c1d < 1.f - p.epsilon_low && A < 0.f) ? 1.f : 0.f;
            const float hi = (c.c1d > 1.f + p.epsilon_high && A > 0.f) ? 1.f : 0.f;
            acc[4] += lo;
            acc[5] += hi;
            acc[6] += fmaxf(lo, hi);
        }
    }
    // Phase 6 (optional): the same metric sums per normaliser segment — one GA
    // micro-batch each — so the host forms the reference's per-micro-batch
    // masked_batch_mean (:2143-2148) before its cross-rank gather.  One wave per
    // segment, rows in index order: fixed summation order.
    if (seg_metrics) {
        for (int s = wid; s < S; s += nw) {
            float sm[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // tok, kl, ent, low, high, region, rows
            for (int64_t r = 0; r < R; ++r) {
                if ((seg ? seg[r] : 0) != s) continue;
                const float A = adv[r];
                const ClipOut cs = clip_term(ws.row_x[r], A, p.epsilon_low, p.epsilon_high, p.delta);
                for (int64_t t = lane; t < T; t += 64) {
                    const int64_t i = r * T + t;
                    const float m = (float)mask[i];
                    sm[0] += m;
                    if (p.beta != 0.f) {
                        const float d = ref[i] - lp[i];
                        sm[1] += (expf(d) - d - 1.f) * m;
                    }
                    if (ent) sm[2] += ent[i] * m;
                    if (!seq) {
                        const ClipOut c = clip_term(old ? lp[i] - old[i] : 0.f, A, p.epsilon_low, p.epsilon_high,
                                                    p.delta);
                        const float lo = (c.c1d < 1.f - p.epsilon_low && A < 0.f) ? 1.f : 0.f;
                        const float hi = (c.c1d > 1.f + p.epsilon_high && A > 0.f) ? 1.f : 0.f;
                        sm[3] += lo * m;
                        sm[4] += hi * m;
                        sm[5] += fmaxf(lo, hi) * m;
                    }
                }
                if (seq && lane == 0) {
                    const float lo = (cs.c1d < 1.f - p.epsilon_low && A < 0.f) ? 1.f : 0.f;
                    const float hi = (cs.c1d > 1.f + p.epsilon_high && A > 0.f) ? 1.f : 0.f;
                    sm[3] += lo;
                    sm[4] += hi;
                    sm[5] += fmaxf(lo, hi);
                }
                if (lane == 0) sm[6] += 1.f;
            }
#pragma unroll
            for (int k = 0; k < 7; ++k) sm[k] = wave_sum(sm[k]);
            if (lane == 0) {
#pragma unroll
                for (int k = 0; k < 7; ++k) seg_metrics[s * 8 + k] = sm[k];
                seg_metrics[s * 8 + 7] = 0.f;
            }
        }
    }
    block_sum<7>(acc, red);
    if (tid == 0) {
        loss[0] = acc[0];
        if (metrics) {
            metrics[0] = acc[1];
            metrics[1] = acc[2];
            metrics[2] = acc[3];
            metrics[3] = acc[4];
            metrics[4] = acc[5];
            metrics[5] = acc[6];
            metrics[6] = (float)R;
            metrics[7] = 0.f;
        }
    }
}

// ---------------------------------------------------------------------------
// a17 — trl/core.py:43-76
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBig) void masked_whiten_kernel(const float *__restrict__ v, const int32_t *__restrict__ m,
                                                             int64_t N, int32_t shift_mean, float *__restrict__ out,
                                                             float *__restrict__ stats) {
    __shared__ double red[2 * (kBig / kWave)];
    double a[2] = {0.0, 0.0};
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) {
        const double mm = (double)m[i];
        a[0] += (double)v[i] * mm;
        a[1] += mm;
    }
    block_sum_d<2>(a, red);
    const double n = a[1];
    const float mean = (float)(a[0] / n);  // masked_mean in the value dtype
    double b[1] = {0.0};
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) {
        const double d = (double)(v[i] - mean);
        b[0] += d * d * (double)m[i];
    }
    block_sum_d<1>(b, red);
    const float var = (float)((b[0] / n) * (n / (n - 1.0)));
    const float rs = 1.0f / sqrtf(var + 1e-8f);
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) {
        float w = (v[i] - mean) * rs;
        if (!shift_mean) w += mean;
        out[i] = w;
    }
    if (threadIdx.x == 0 && stats) {
        stats[0] = mean;
        stats[1] = var;
        stats[2] = (float)n;
    }
}

// ---------------------------------------------------------------------------
// a18 — ppo_trainer.py:523-535 (one thread per row, reverse recursion)
// ---------------------------------------------------------------------------
__global__ void gae_kernel(const float *__restrict__ rw, const float *__restrict__ val, int64_t B, int64_t T,
                           float gamma, float lam, float *__restrict__ adv, float *__restrict__ ret) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    float last = 0.f;
    for (int64_t t = T - 1; t >= 0; --t) {
        const float nv = (t < T - 1) ? val[b * T + t + 1] : 0.f;
        const float v = val[b * T + t];
        const float delta = rw[b * T + t] + gamma * nv - v;
        last = delta + gamma * lam * last;
        adv[b * T + t] = last;
        ret[b * T + t] = last + v;
    }
}

// ---------------------------------------------------------------------------
// a19 — ppo_trainer.py:557-605
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBig) void ppo_loss_kernel(
    const float *__restrict__ nl, const float *__restrict__ ol, const float *__restrict__ adv,
    const float *__restrict__ vp, const float *__restrict__ ov, const float *__restrict__ ret,
    const uint8_t *__restrict__ pm, const uint8_t *__restrict__ pm1, int64_t N, float cr, float cv, float vf_coef,
    float *__restrict__ loss, float *__restrict__ dnl, float *__restrict__ dvp, float *__restrict__ stats) {
    __shared__ float red[8 * (kBig / kWave)];
    // pass 1: mask counts
    float c[2] = {0.f, 0.f};
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) {
        c[0] += pm[i] ? 0.f : 1.f;
        c[1] += pm1[i] ? 0.f : 1.f;
    }
    block_sum<2>(c, red);
    const float n_pg = c[0], n_vf = c[1];
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // pg, vf, pgclip, vfclip, kl, ratio
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) {
        const float A = adv[i];
        const float diff = nl[i] - ol[i];
        const float ratio = expf(diff);
        const float rc = fminf(fmaxf(ratio, 1.f - cr), 1.f + cr);
        const float p1 = -A * ratio, p2 = -A * rc;
        const float kp = pm[i] ? 0.f : 1.f;
        a[0] += fmaxf(p1, p2) * kp;
        a[2] += (p2 > p1 ? 1.f : 0.f) * kp;
        if (dnl) {
            float g1, g2;
            if (p1 > p2) { g1 = 1.f; g2 = 0.f; }
            else if (p2 > p1) { g1 = 0.f; g2 = 1.f; }
            else { g1 = 0.5f; g2 = 0.5f; }
            const float dp1 = -A * ratio;
            const float dp2 = -A * ratio * ((ratio >= 1.f - cr && ratio <= 1.f + cr) ? 1.f : 0.f);
            dnl[i] = kp * (g1 * dp1 + g2 * dp2) / n_pg;
        }
        const float v = vp[i], o = ov[i], R = ret[i];
        const float vcl = fminf(fmaxf(v, o - cv), o + cv);
        const float v1 = (v - R) * (v - R), v2 = (vcl - R) * (vcl - R);
        const float kv = pm1[i] ? 0.f : 1.f;
        a[1] += fmaxf(v1, v2) * kv;
        a[3] += (v2 > v1 ? 1.f : 0.f) * kv;
        if (dvp) {
            float g1, g2;
            if (v1 > v2) { g1 = 1.f; g2 = 0.f; }
            else if (v2 > v1) { g1 = 0.f; g2 = 1.f; }
            else { g1 = 0.5f; g2 = 0.5f; }
            const float dv1 = 2.f * (v - R);
            const float dv2 = 2.f * (vcl - R) * ((v >= o - cv && v <= o + cv) ? 1.f : 0.f);
            dvp[i] = kv * vf_coef * 0.5f * (g1 * dv1 + g2 * dv2) / n_vf;
        }
        a[4] += diff * diff;
        a[5] += ratio;
    }
    block_sum<8>(a, red);
    if (threadIdx.x == 0) {
        const float pg = a[0] / n_pg, vf = 0.5f * (a[1] / n_vf);
        loss[0] = pg + vf_coef * vf;
        if (stats) {
            stats[0] = pg;
            stats[1] = vf;
            stats[2] = a[2] / n_pg;
            stats[3] = a[3] / n_vf;
            stats[4] = 0.5f * (a[4] / (float)N);
            stats[5] = a[5] / (float)N;
            stats[6] = 0.f;
            stats[7] = 0.f;
        }
    }
}

// ---------------------------------------------------------------------------
// a20 — modeling_value_head.py:50-59 / score head (one wave per row)
// ---------------------------------------------------------------------------
template <int DT>
__global__ __launch_bounds__(256) void value_head_kernel(const typename Elem<DT>::T *__restrict__ h, int64_t R,
                                                         int64_t H, int64_t ld, const float *__restrict__ w,
                                                         const float *__restrict__ bias, float *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= R) return;
    float s = 0.f;
    for (int64_t k = lane; k < H; k += 64) s += Elem<DT>::load(h + r * ld + k) * w[k];
    s = wave_sum(s);
    if (lane == 0) out[r] = s + (bias ? bias[0] : 0.f);
}


// ---------------------------------------------------------------------------
// a16 — PPO rollout post-processing (ppo_trainer.py:478-516), one workgroup
// per row: (1) truncate_response after the first stop token and the sequence
// length (first pad of the truncated row, minus one: utils.py:1036-1056,
// :877-897); (2) the masks, INVALID_LOGPROB fill, value masking, missing-EOS
// penalty, k1/k3 KL, KL-shaped rewards and the score scatter at
// min(seq_len + 1, T - 1).  Replaces ~15 torch launches of host glue.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int block_min_i32(int v, int *red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, kWave));
    if (lane == 0) red[wid] = v;
    __syncthreads();
    int r = red[0];
    for (int w = 1; w < nw; ++w) r = min(r, red[w]);
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(256) void ppo_truncate_kernel(const int64_t *__restrict__ resp, int64_t T,
                                                           int64_t stop, int64_t pad, int64_t *__restrict__ post,
                                                           int64_t *__restrict__ seq_len) {
    __shared__ int red[4];
    const int64_t b = blockIdx.x;
    const int64_t *r = resp + b * T;
    int first = (int)T;
    if (stop >= 0)
        for (int64_t t = threadIdx.x; t < T; t += blockDim.x)
            if (r[t] == stop) { first = (int)t; break; }
    first = block_min_i32(first, red);
    int fpad = (int)T;
    for (int64_t t = threadIdx.x; t < T; t += blockDim.x) {
        const int64_t v = (t > first) ? pad : r[t];
        post[b * T + t] = v;
        if (v == pad && (int)t < fpad) fpad = (int)t;
    }
    fpad = block_min_i32(fpad, red);
    if (threadIdx.x == 0) seq_len[b] = (int64_t)fpad - 1;
}

// DT: dtype of the score heads' outputs (values / scores): bf16 for the bf16
// engine, f32 in the reference-precision mode; every update rounds like the
// reference's tensor of that dtype.
template <int DT>
__global__ __launch_bounds__(256) void ppo_rewards_kernel(
    const int64_t *__restrict__ post, const int64_t *__restrict__ seq_len, int64_t T, int64_t eos, float penalty,
    int32_t has_penalty, float kl_coef, int32_t k3, float *__restrict__ logp, float *__restrict__ ref,
    typename Elem<DT>::T *__restrict__ values, typename Elem<DT>::T *__restrict__ scores, uint8_t *__restrict__ pmask,
    uint8_t *__restrict__ pmask1, float *__restrict__ kl, float *__restrict__ nsr, float *__restrict__ rewards) {
    __shared__ int red[4];
    const int64_t b = blockIdx.x;
    const int64_t sl = seq_len[b];
    int has = 0;
    if (eos >= 0)
        for (int64_t t = threadIdx.x; t < T; t += blockDim.x) has |= (post[b * T + t] == eos);
    has = -block_min_i32(-has, red);  // any
    float score = Elem<DT>::load(scores + b);
    if (has_penalty && !has) score = Elem<DT>::round(score - penalty);  // the score tensor minus a Python float
    const int64_t end = (sl + 1 < T) ? sl + 1 : sl;                  // ppo_trainer.py:513-515
    for (int64_t t = threadIdx.x; t < T; t += blockDim.x) {
        const int64_t i = b * T + t;
        const bool pm = t > sl, pm1 = t > sl + 1;
        pmask[i] = pm;
        pmask1[i] = pm1;
        const float lp = pm ? 1.0f : logp[i];  // INVALID_LOGPROB (ppo_trainer.py:81)
        const float rf = pm ? 1.0f : ref[i];
        logp[i] = lp;
        ref[i] = rf;
        if (pm1) values[i] = 0;
        const float logr = rf - lp;
        const float k = k3 ? (expf(logr) - 1.f) - logr : -logr;
        const float n = -kl_coef * k;
        kl[i] = k;
        nsr[i] = n;
        rewards[i] = (t == end) ? n + score : n;
    }
    if (threadIdx.x == 0) {
        if constexpr (DT == SWH_F32) scores[b] = score;
        else scores[b] = f32_to_bf16_bits(score);
    }
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int swh_completion_mask(const int64_t *ids, int64_t B, int64_t C, const int32_t *eos_ids, int32_t n_eos,
                                   int32_t mask_truncated, int32_t *mask, int32_t *lengths, int32_t *has_eos,
                                   void *stream) {
    if (!ids || !mask || B < 0 || C < 0 || n_eos < 0 || (n_eos > 0 && !eos_ids)) return SWH_E_ARG;
    if (B == 0 || C == 0) return SWH_OK;
    completion_mask_kernel<<<dim3((unsigned)B), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(
        ids, C, eos_ids, n_eos, mask_truncated, mask, lengths, has_eos);
    return launch_status();
}

extern "C" int swh_group_advantage(const float *rpf, const float *w, int64_t N, int64_t F, int64_t G,
                                   int32_t scale_rewards, float *advantages, float *rewards, float *group_mean,
                                   float *group_std, int32_t *zero_std, void *stream) {
    if (!rpf || !w || !advantages || N < 0 || F <= 0 || G < 2 || N % G != 0) return SWH_E_ARG;
    if (N == 0) return SWH_OK;
    const int64_t ng = N / G;
    group_advantage_kernel<<<dim3((unsigned)((ng + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(
        rpf, w, N, F, G, scale_rewards, advantages, rewards, group_mean, group_std, zero_std);
    return launch_status();
}

extern "C" int64_t swh_grpo_loss_workspace_bytes(int64_t R) { return (4 * R + 2 * 4096 + 64) * 4; }

extern "C" int swh_grpo_loss_fwd_bwd(const float *logp, const float *old_logp, const float *ref_logp,
                                     const float *adv, const int32_t *mask, const uint8_t *ent_mask,
                                     const float *entropy, const float *row_scale, const int32_t *seg, int64_t R,
                                     int64_t T, const swh_grpo_loss_params *p, float *loss, float *dlogp,
                                     float *metrics, float *seg_metrics, void *workspace, void *stream) {
    if (!logp || !adv || !mask || !p || !loss || !workspace || R <= 0 || T <= 0) return SWH_E_ARG;
    const swh_grpo_loss_params pp = *p;
    if (pp.num_segments < 1 || pp.num_segments > 4096 || pp.loss_type < 0 || pp.loss_type > 2 || pp.is_level < 0 ||
        pp.is_level > 1 || (pp.beta != 0.f && !ref_logp) || (pp.num_segments > 1 && !seg))
        return SWH_E_ARG;
    if (pp.loss_type == SWH_LOSS_DR_GRPO && pp.max_completion_length <= 0) return SWH_E_ARG;
    float *w = static_cast<float *>(workspace);
    LossWS ws{w, w + R, w + 2 * R, w + 3 * R, w + 4 * R, w + 4 * R + 4096};
    grpo_loss_kernel<<<1, kBig, 0, static_cast<hipStream_t>(stream)>>>(logp, old_logp, ref_logp, adv, mask, ent_mask,
                                                                     entropy, row_scale, seg, R, T, pp, loss, dlogp,
                                                                     metrics, seg_metrics, ws);
    return launch_status();
}

extern "C" int64_t swh_masked_whiten_workspace_bytes(int64_t N) {
    (void)N;
    return 0;
}

extern "C" int swh_masked_whiten(const float *values, const int32_t *mask, int64_t N, int32_t shift_mean, float *out,
                                 float *stats, void *workspace, void *stream) {
    (void)workspace;
    if (!values || !mask || !out || N <= 0) return SWH_E_ARG;
    masked_whiten_kernel<<<1, kBig, 0, static_cast<hipStream_t>(stream)>>>(values, mask, N, shift_mean, out, stats);
    return launch_status();
}

extern "C" int swh_gae_scan(const float *rewards, const float *values, int64_t B, int64_t T, float gamma, float lam,
                            float *advantages, float *returns, void *stream) {
    if (!rewards || !values || !advantages || !returns || B < 0 || T < 0) return SWH_E_ARG;
    if (B == 0 || T == 0) return SWH_OK;
    gae_kernel<<<dim3((unsigned)((B + 63) / 64)), dim3(64), 0, static_cast<hipStream_t>(stream)>>>(
        rewards, values, B, T, gamma, lam, advantages, returns);
    return launch_status();
}

extern "C" int64_t swh_ppo_loss_workspace_bytes(int64_t N) {
    (void)N;
    return 0;
}

extern "C" int swh_ppo_loss_fwd_bwd(const float *new_logp, const float *old_logp, const float *adv, const float *vpred,
                                    const float *old_values, const float *returns, const uint8_t *pad_mask,
                                    const uint8_t *pad_mask_p1, int64_t B, int64_t T, float cliprange,
                                    float cliprange_value, float vf_coef, float *loss, float *dnew_logp, float *dvpred,
                                    float *stats, void *workspace, void *stream) {
    (void)workspace;
    if (!new_logp || !old_logp || !adv || !vpred || !old_values || !returns || !pad_mask || !pad_mask_p1 || !loss ||
        B <= 0 || T <= 0)
        return SWH_E_ARG;
    ppo_loss_kernel<<<1, kBig, 0, static_cast<hipStream_t>(stream)>>>(new_logp, old_logp, adv, vpred, old_values,
                                                                    returns, pad_mask, pad_mask_p1, B * T, cliprange,
                                                                    cliprange_value, vf_coef, loss, dnew_logp, dvpred,
                                                                    stats);
    return launch_status();
}

extern "C" int swh_value_head_fwd(const void *hidden, int dtype, int64_t R, int64_t H, int64_t ld, const float *w,
                                  const float *bias, float *out, void *stream) {
    if (!hidden || !w || !out || R < 0 || H <= 0 || ld < H) return SWH_E_ARG;
    if (R == 0) return SWH_OK;
    dim3 grid((unsigned)((R + 3) / 4)), block(256);
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
    case SWH_BF16:
        value_head_kernel<SWH_BF16><<<grid, block, 0, s>>>(static_cast<const uint16_t *>(hidden), R, H, ld, w, bias, out);
        break;
    case SWH_F32:
        value_head_kernel<SWH_F32><<<grid, block, 0, s>>>(static_cast<const float *>(hidden), R, H, ld, w, bias, out);
        break;
    default:
        return SWH_E_DTYPE;
    }
    return launch_status();
}

extern "C" int swh_ppo_truncate(const int64_t *responses, int64_t B, int64_t T, int64_t stop_token_id,
                                int64_t pad_token_id, int64_t *post, int64_t *seq_len, void *stream) {
    if (!responses || !post || !seq_len || B < 0 || T <= 0 || T > (1 << 30)) return SWH_E_ARG;
    if (B == 0) return SWH_OK;
    ppo_truncate_kernel<<<dim3((unsigned)B), 256, 0, static_cast<hipStream_t>(stream)>>>(responses, T, stop_token_id,
                                                                                          pad_token_id, post, seq_len);
    return launch_status();
}

extern "C" int swh_ppo_rewards(const int64_t *post, const int64_t *seq_len, int64_t B, int64_t T, int64_t eos_token_id,
                               float missing_eos_penalty, int32_t has_penalty, float kl_coef, int32_t kl_k3,
                               float *logprobs, float *ref_logprobs, void *values, void *scores, int32_t dtype,
                               uint8_t *padding_mask, uint8_t *padding_mask_p1, float *kl, float *non_score_reward,
                               float *rewards, void *stream) {
    if (!post || !seq_len || !logprobs || !ref_logprobs || !values || !scores || !padding_mask ||
        !padding_mask_p1 || !kl || !non_score_reward || !rewards || B < 0 || T <= 0 || T > (1 << 30) ||
        (dtype != SWH_F32 && dtype != SWH_BF16))
        return SWH_E_ARG;
    if (B == 0) return SWH_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (dtype == SWH_F32)
        ppo_rewards_kernel<SWH_F32><<<dim3((unsigned)B), 256, 0, s>>>(
            post, seq_len, T, eos_token_id, missing_eos_penalty, has_penalty, kl_coef, kl_k3, logprobs, ref_logprobs,
            static_cast<float *>(values), static_cast<float *>(scores), padding_mask, padding_mask_p1, kl,
            non_score_reward, rewards);
    else
        ppo_rewards_kernel<SWH_BF16><<<dim3((unsigned)B), 256, 0, s>>>(
            post, seq_len, T, eos_token_id, missing_eos_penalty, has_penalty, kl_coef, kl_k3, logprobs, ref_logprobs,
            static_cast<uint16_t *>(values), static_cast<uint16_t *>(scores), padding_mask, padding_mask_p1, kl,
            non_score_reward, rewards);
    return launch_status();
}
