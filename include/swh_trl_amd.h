/*
 * swh_trl_amd — C-ABI of the MI355X-native GRPO/PPO rollout-and-update hot path.
 *
 * Every entry point is a stream-ordered device launch:
 *   - all pointers are CALLER-OWNED DEVICE buffers (allocated by PyTorch in the
 *     host layer); scratch comes in as an explicit workspace argument — the
 *     library never calls hipMalloc, never synchronises, never copies to host;
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream);
 *   - return value: 0 = launched, <0 = error (see SWH_E_*); argument errors are
 *     detected on the host before anything is launched;
 *   - no hidden mutable state: the library holds only (1) per-device facts
 *     queried once per device under std::call_once (CU count, each kernel's
 *     dynamic-LDS opt-in) and (2) the launch policy below, one per host thread
 *     (thread_local), set explicitly by swh_set_launch_policy; nothing is
 *     process-wide and mutable, and it never reads the environment.  Entry
 *     points are re-entrant across host threads, streams
 *     and devices, and safe to capture into a hipGraph (the decode step is
 *     captured and replayed).
 *
 * Each function cites the reference (shiwanghua/swh-trl @ TRL 0.21.0.dev0)
 * symbol it replaces, `path:line` relative to the reference tree.
 * Dtype codes: SWH_F32 = 0, SWH_BF16 = 1, SWH_F16 = 2.
 */
#ifndef SWH_TRL_AMD_H
#define SWH_TRL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWH_OK 0
#define SWH_E_ARG (-1)      /* invalid argument (shape, dtype, null pointer) */
#define SWH_E_LAUNCH (-2)   /* hipGetLastError() after the launch was not hipSuccess */
#define SWH_E_DTYPE (-3)    /* dtype not supported by this entry point */

#define SWH_F32 0
#define SWH_BF16 1
#define SWH_F16 2

/* ---- library ------------------------------------------------------------ */
const char *swh_version(void);
const char *swh_status_string(int status);

/* Launch policy: geometry choices of the decode GEMMs and samplers, for A/B
 * timing and geometry-coverage tests.  Every alternative is bit-identical
 * (tests pin that) except wide_smax, wide_cb and wide_waves, which choose how
 * wide_gemm splits K, and attn_pair, which chooses how the D = 128 decode
 * attention's waves split the keys: these change the fp32 summation order
 * (each deterministic for a given policy).  Per host thread: a thread's policy
 * starts at the defaults and applies to the launches that thread issues after
 * the call (a captured graph keeps the geometry it was captured with); other
 * threads are not affected.  *_workspace_bytes size for the policy in force when they are
 * called; a launch whose geometry needs more workspace than it is given returns
 * SWH_E_ARG and writes nothing.  gemm_ms 0 means "the cost model decides" (the
 * other geometry fields must then be 0). */
typedef struct swh_launch_policy {
    int64_t wide_kmin;     /* smallest K routed to the bandwidth-regime GEMM (csrc/wide_gemm.hip); 2048 */
    int32_t wide_gemm;     /* 0: every decode projection on decode_gemm; 1 */
    int32_t wide_smax;     /* largest K split of wide_gemm, 1..8; 8 */
    int32_t wide_cb;       /* 16-row weight groups per wave of wide_gemm: 0 auto, 1, 2; 0 */
    int32_t gemm_ms;       /* decode_gemm geometry override: 16-row blocks 1/2/4 (0 = cost model), */
    int32_t gemm_cb;       /*   16-column blocks 1/2/4, */
    int32_t gemm_s;        /*   K split 1..8, */
    int32_t gemm_persist;  /*   persistent grid 0/1, */
    int32_t gemm_wn;       /*   column groups 1/2/4; */
    int32_t gemm_tile;     /* 1: force the tile kernel where it applies; 0 */
    int32_t gemm_nw;       /* waves per decode_gemm workgroup 4/8/16 (0 = 8); 0 */
    int32_t xstream;       /* 0: qkv / o through decode_gemm's LDS X image instead of register-streamed X; 1 */
    int32_t lm_ring14;     /* 0: whole-tile weight ring in the fused lm-head sampler at K = 896; 1 */
    int32_t filt_wgs;      /* target workgroups of one filtered-sampler pass, 64..65536; 1024 */
    int32_t wide_waves;    /* waves per 128-row-class wide_gemm workgroup (16 x waves weight rows):
                            * 0 auto (the count that fills the CUs best), 6, 7, 8; 0 */
    int32_t attn_pair;     /* 1: decode attention at D = 128 on one workgroup per (kv head, two rows),
                            * a shared GRPO prompt's keys read once for both; 0: one per row; 1 */
} swh_launch_policy;
int swh_launch_policy_default(swh_launch_policy *out);
int swh_get_launch_policy(swh_launch_policy *out);
int swh_set_launch_policy(const swh_launch_policy *p);  /* SWH_E_ARG when a field is out of range */

/* ---- a6/a7/a8: log-probs + entropy of temperature-scaled logits ----------
 * Replaces trl/trainer/utils.py:1430-1462 (selective_log_softmax),
 * :1465-1490 (entropy_from_logits) and the `logits / self.temperature` of
 * grpo_trainer.py:1254 / ppo_trainer.py:446,558.
 * Rows are addressed as r = o*rows_inner + i with element offset
 * o*stride_outer + i*stride_inner (lets the caller pass the [:, -C-1:-1]
 * slice of a [B, L, V] logits tensor without a copy).  ids/logp/entropy/lse
 * are contiguous [rows_outer*rows_inner].  z = logits / temperature.
 *   logp[r]    = z[r, ids[r]] - logsumexp(z[r, :])
 *   entropy[r] = -sum_j p_j log p_j          (entropy may be NULL)
 *   lse[r]     = logsumexp(z[r, :])          (saved for the backward)
 * flags: SWH_LOGP_ROUND_SCALED — round z to the logits dtype after the
 * division, as the reference does when it divides bf16 logits in bf16. */
#define SWH_LOGP_ROUND_SCALED 1
int swh_logp_entropy_fwd(const void *logits, int dtype, int64_t rows_outer, int64_t rows_inner,
                         int64_t stride_outer, int64_t stride_inner, int64_t V, const int64_t *ids,
                         float temperature, int flags, float *logp, float *entropy, float *lse,
                         void *stream);

/* Backward of logp w.r.t. the logits (autograd of selective_log_softmax and
 * of the temperature division): dlogits[r, j] = dlogp[r]/T * (1[j==ids[r]] - p_j).
 * dlogits has the logits dtype and its own (outer, inner) strides; row
 * stride between elements is 1. */
int swh_logp_bwd(const void *logits, int dtype, int64_t rows_outer, int64_t rows_inner,
                 int64_t stride_outer, int64_t stride_inner, int64_t V, const int64_t *ids,
                 float temperature, int flags, const float *lse, const float *dlogp, void *dlogits,
                 int64_t dstride_outer, int64_t dstride_inner, void *stream);
/* selective_log_softmax for bf16/fp16 rows of V <= 1024 (trl/trainer/utils.py:1451-1459,
 * the half-precision `log_softmax(row).gather` branch): the fp32 operations of
 * torch's persistent warp softmax in its order, so out (logits dtype, [rows])
 * equals torch.gather(logits.log_softmax(-1), -1, ids) bit for bit
 * (tests/test_utils.py:540-558).  SWH_E_ARG for V > 1024, SWH_E_DTYPE for f32. */
int swh_log_softmax_gather_exact(const void *logits, int dtype, int64_t rows_outer, int64_t rows_inner,
                                 int64_t stride_outer, int64_t stride_inner, int64_t V, const int64_t *ids,
                                 void *out, void *stream);


/* ---- a4: one rollout sampling step ----------------------------------------
 * Replaces the HF `_sample` body the reference reaches through
 * grpo_trainer.py:1793-1810 (processors built from GenerationConfig
 * :995-1014): repetition penalty -> min-new-tokens EOS suppression ->
 * temperature -> top-k -> top-p -> min-p, then an exact categorical draw
 * (Gumbel-max over a Philox4x32-10 stream) or argmax,
 * then pad-after-EOS bookkeeping.  All step-dependent state lives on the
 * device so the call can be graph-captured and replayed.
 *   logits      [B, V] (row stride ld), dtype bf16/f32
 *   rng         device uint64[2] = {seed (Philox key), counter base}; the
 *               counter of token t is base + t, so a replayed graph draws
 *               fresh numbers when the host bumps rng[1] between rollouts
 *   step        device int32: index of the token being generated
 *   finished    device int32 [B]  (in/out)
 *   seen        device uint32 [B, ceil(V/32)] membership bitmap for the
 *               repetition penalty (in/out; may be NULL when penalty == 1)
 *   out_tokens  int64 [B, out_ld]; token written at column *step
 *   cur_tokens  int64 [B]; the same token (next decode input)
 *   out_logp    f32 [B, out_ld] or NULL: log-prob of the drawn token under the
 *               processed distribution (the PPO rollout log-prob, utils.py:1094)
 *   scores_out  f32 [B, V] or NULL: processed scores (HF output_scores)
 *   workspace   >= swh_sample_workspace_bytes(B, V) bytes: split partials, and
 *               for filtered rows their threshold state and per-split digit
 *               histograms (the filtered path is several launches on `stream`) */
typedef struct {
    float temperature;        /* 1.0 = off */
    float top_p;              /* 1.0 = off */
    float min_p;              /* <= 0 = off */
    float repetition_penalty; /* 1.0 = off */
    int32_t top_k;            /* 0 = off */
    int32_t greedy;           /* 1 = argmax (do_sample=False) */
    int32_t min_new_tokens;   /* EOS suppressed while *step < min_new_tokens */
    int32_t pad_token_id;     /* emitted by finished rows; -1 = no pad bookkeeping */
    int32_t n_eos;            /* number of valid eos ids (0..4) */
    int32_t eos_ids[4];
} swh_sample_params;
int64_t swh_sample_workspace_bytes(int64_t B, int64_t V);
int swh_sample_step(const void *logits, int dtype, int64_t B, int64_t V, int64_t ld,
                    const swh_sample_params *params, const uint64_t *rng, const int32_t *step,
                    int32_t *finished,
                    uint32_t *seen, int64_t *out_tokens, int64_t out_ld, int64_t *cur_tokens,
                    float *out_logp, float *scores_out, void *workspace, void *stream);
/* Sets the `seen` bitmap from prompt ids (ids < 0 or mask == 0 are skipped). */
int swh_seen_init(const int64_t *ids, const int32_t *mask, int64_t B, int64_t L, int64_t V,
                  uint32_t *seen, void *stream);
/* Increments the device step counter (end of a captured decode step). */
int swh_step_advance(int32_t *step, void *stream);

/* ---- a5: completion mask ---------------------------------------------------
 * Replaces grpo_trainer.py:1812-1831: mask[b,t] = t <= first EOS (EOS
 * included), lengths[b] = sum_t mask, has_eos[b]; rows with no EOS are zeroed
 * when mask_truncated != 0. */
int swh_completion_mask(const int64_t *completion_ids, int64_t B, int64_t C, const int32_t *eos_ids,
                        int32_t n_eos, int32_t mask_truncated, int32_t *mask, int32_t *lengths,
                        int32_t *has_eos, void *stream);

/* ---- a10: group-relative advantages -----------------------------------------
 * Replaces grpo_trainer.py:1914-1930: r = nansum_f(rpf*w); per group of G
 * rows mean and UNBIASED std; A = r - mean, /(std + 1e-4) if scale_rewards;
 * zero_std[g] = isclose(std, 0).  Any of group_mean/group_std/zero_std/
 * rewards may be NULL. */
int swh_group_advantage(const float *rewards_per_func, const float *weights, int64_t N, int64_t F,
                        int64_t G, int32_t scale_rewards, float *advantages, float *rewards,
                        float *group_mean, float *group_std, int32_t *zero_std, void *stream);

/* ---- a11: GRPO policy loss, forward + d loss / d logp in one pass -----------
 * Replaces grpo_trainer.py:2058-2175 from the log-probs on: k3 KL (:2085),
 * token/sequence importance weights (:2099-2111), two-sided clip and delta
 * (:2113-2118), -min(c1 A, c2 A) (:2120), entropy mask (:2123), +beta KL
 * (:2125), grpo/bnpo/dr_grpo aggregation (:2130-2137), and the metric sums
 * behind :2139-2174.  Gradient conventions follow torch autograd exactly
 * (min ties split 1/2-1/2, clamp passes the gradient on the closed interval).
 *   logp/old/ref f32 [R, T] (old/ref nullable; old NULL == logp.detach())
 *   adv f32 [R]; mask int32 [R, T]; ent_mask uint8 [R, T] nullable;
 *   entropy f32 [R, T] nullable (metrics only); row_scale f32 [R] nullable:
 *   extra per-row loss weight (used to fuse gradient-accumulation micro-
 *   batches into one pass; NULL = 1).  seg [R] int32 nullable: normaliser
 *   segment of each row (bnpo token counts are per segment; NULL = one).
 * Outputs: loss f32[1] (sum over segments of each segment's loss, times
 * row_scale), dlogp f32 [R, T] (d loss / d logp, may be NULL), metrics f32[8]:
 * {tokens, kl_sum, entropy_sum, low_clip_sum, high_clip_sum, region_clip_sum,
 *  seq_rows, 0}; seg_metrics f32 [num_segments, 8] nullable: the same sums
 * per segment (clip sums over rows under sequence level, last-but-one = rows),
 * from which the host forms each micro-batch's masked_batch_mean
 * (:2143-2148) before the cross-rank gather (:2150-2174).
 * workspace >= swh_grpo_loss_workspace_bytes(R). */
#define SWH_LOSS_GRPO 0
#define SWH_LOSS_BNPO 1
#define SWH_LOSS_DR_GRPO 2
#define SWH_IS_TOKEN 0
#define SWH_IS_SEQUENCE 1
typedef struct {
    float beta;
    float epsilon_low;
    float epsilon_high;
    float delta;              /* <= 0 = off */
    int32_t loss_type;        /* SWH_LOSS_* */
    int32_t is_level;         /* SWH_IS_* */
    int32_t max_completion_length;
    int32_t num_segments;     /* >= 1 */
} swh_grpo_loss_params;
int64_t swh_grpo_loss_workspace_bytes(int64_t R);
int swh_grpo_loss_fwd_bwd(const float *logp, const float *old_logp, const float *ref_logp,
                          const float *adv, const int32_t *mask, const uint8_t *ent_mask,
                          const float *entropy, const float *row_scale, const int32_t *seg, int64_t R,
                          int64_t T, const swh_grpo_loss_params *p, float *loss, float *dlogp,
                          float *metrics, float *seg_metrics, void *workspace, void *stream);

/* ---- a17: masked mean / var / whiten (trl/core.py:43-76) -----------------
 * values f32 [N], mask int32 [N]; out f32 [N]; stats f32[3] = {mean, var,
 * mask_sum}.  A zero mask sum yields NaN stats (the host raises ValueError
 * like core.py:59).  workspace >= swh_masked_whiten_workspace_bytes(N). */
int64_t swh_masked_whiten_workspace_bytes(int64_t N);
int swh_masked_whiten(const float *values, const int32_t *mask, int64_t N, int32_t shift_mean,
                      float *out, float *stats, void *workspace, void *stream);

/* ---- a18: GAE reverse scan (ppo_trainer.py:523-535) --------------------
 * rewards/values f32 [B, T] -> advantages, returns f32 [B, T]. */
int swh_gae_scan(const float *rewards, const float *values, int64_t B, int64_t T, float gamma,
                 float lam, float *advantages, float *returns, void *stream);

/* ---- a19: PPO clipped policy + value loss, fwd + bwd (ppo_trainer.py:557-605)
 * new_logp, old_logp, adv, vpred, old_values, returns f32 [B, T];
 * pad_mask / pad_mask_p1 uint8 [B, T] (1 = padding, as the reference's
 * padding_mask / padding_mask_p1).  Outputs: loss f32[1],
 * dnew_logp / dvpred f32 [B,T] (nullable), stats f32[8] =
 * {pg_loss, vf_loss, pg_clipfrac, vf_clipfrac, approxkl, ratio_mean, 0, 0}.
 * workspace >= swh_ppo_loss_workspace_bytes(B*T). */
int64_t swh_ppo_loss_workspace_bytes(int64_t N);
int swh_ppo_loss_fwd_bwd(const float *new_logp, const float *old_logp, const float *adv,
                         const float *vpred, const float *old_values, const float *returns,
                         const uint8_t *pad_mask, const uint8_t *pad_mask_p1, int64_t B, int64_t T,
                         float cliprange, float cliprange_value, float vf_coef, float *loss,
                         float *dnew_logp, float *dvpred, float *stats, void *workspace, void *stream);

/* ---- a16: PPO rollout post-processing (ppo_trainer.py:478-516) --------------
 * swh_ppo_truncate: post = truncate_response(stop, pad, responses) (utils.py
 * :1036-1056: tokens after the first stop token become pad; stop < 0 = none),
 * seq_len[b] = first_true_indices(post == pad) - 1 (utils.py:877-897).
 * responses / post int64 [B, T]; seq_len int64 [B]. */
int swh_ppo_truncate(const int64_t *responses, int64_t B, int64_t T, int64_t stop_token_id, int64_t pad_token_id,
                     int64_t *post, int64_t *seq_len, void *stream);
/* swh_ppo_rewards, per row after the value / reward-model forwards:
 * padding_mask = t > seq_len, padding_mask_p1 = t > seq_len + 1 (uint8 [B, T]);
 * logprobs / ref_logprobs f32 [B, T] set to INVALID_LOGPROB (1.0) under the
 * mask (in place); values [B, T] zeroed under mask_p1 (in place); scores [B]
 * minus missing_eos_penalty where no eos token is in post (has_penalty, eos < 0
 * = none; in place, rounded to their dtype); values / scores are the score
 * heads' outputs in `dtype` (SWH_BF16, or SWH_F32 in the reference-precision
 * mode); kl = -logr (k1) or (exp(logr) - 1) - logr (k3), logr = ref - logp;
 * non_score_reward = -kl_coef * kl; rewards = non_score_reward + score at
 * min(seq_len + 1, T - 1) (all f32 [B, T]). */
int swh_ppo_rewards(const int64_t *post, const int64_t *seq_len, int64_t B, int64_t T, int64_t eos_token_id,
                    float missing_eos_penalty, int32_t has_penalty, float kl_coef, int32_t kl_k3, float *logprobs,
                    float *ref_logprobs, void *values, void *scores, int32_t dtype, uint8_t *padding_mask,
                    uint8_t *padding_mask_p1, float *kl, float *non_score_reward, float *rewards, void *stream);

/* ---- a20: value head (modeling_value_head.py:50-59; PPO score head
 * ppo_trainer.py:95, utils.py:937): out[r] = sum_h hidden[r,h]*w[h] (+ bias).
 * hidden bf16/f32 [R, H] row stride ld; w f32 [H]; bias nullable f32[1]. */
int swh_value_head_fwd(const void *hidden, int dtype, int64_t R, int64_t H, int64_t ld, const float *w,
                       const float *bias, float *out, void *stream);

/* ---- a13: optimizer --------------------------------------------------------
 * Squared-L2 partial sums of a flat gradient buffer: partials f32
 * [swh_sqnorm_partials(N)]; then swh_finalize_clip reduces them to the total
 * norm and the clip coefficient min(1, max_norm/(norm+1e-6)) on device
 * (torch.nn.utils.clip_grad_norm_ semantics; max_norm <= 0 => coef 1).
 * out2 f32[2] = {total_norm, clip_coef}. */
int64_t swh_sqnorm_partials(int64_t N);
int swh_grad_sqnorm(const void *grad, int dtype, int64_t N, float *partials, void *stream);
int swh_finalize_clip(const float *partials, int64_t n_partials, float max_norm, float *out2,
                      void *stream);
/* Decoupled AdamW over flat buffers (torch.optim.AdamW update rule):
 *   g = grad * clip[1] (clip NULL => 1) ; p *= 1 - lr*wd ;
 *   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ;
 *   p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
 * master/m/v f32 [N]; grad bf16/f32 [N]; model_out [N] of model_dtype (bf16:
 * the refreshed low-precision weights; f32: an fp32 model's own weights) or
 * NULL; step_count >= 1.  no_decay int64 [2 n_no_decay] = sorted, disjoint
 * [start, end) element ranges updated with weight_decay 0 (transformers
 * Trainer.get_decay_parameter_names: biases and norm weights), each start/end
 * a multiple of 4; NULL / 0 = decay everywhere. */
int swh_adamw(float *master, float *exp_avg, float *exp_avg_sq, const void *grad, int grad_dtype,
              void *model_out, int model_dtype, int64_t N, float lr, float beta1, float beta2, float eps,
              float weight_decay, int64_t step_count, const float *clip, const int64_t *no_decay,
              int32_t n_no_decay, void *stream);
/* TR-DPO reference-model sync (trl/trainer/callbacks.py:106-131, SyncRefModelCallback
 * ._sync_target_model, run every ref_model_sync_steps by grpo_trainer.py:1032-1033):
 * target = target * keep + alpha * src over a flat parameter buffer, keep =
 * float(1 - alpha) formed by the caller in double precision (torch casts the
 * Python scalar 1 - alpha), rounded to the parameter dtype after the multiply and
 * after the add as torch's mul_ / add_(alpha=) do.  dtype bf16 or f32. */
int swh_ema_mix(void *target, const void *src, int dtype, int64_t N, float keep, float alpha, void *stream);
/* Token-split weight gradient fold (the training backward's dW = dY^T X split
 * over S token ranges into a batched GEMM): grad[i] = round(grad[i] +
 * sum_s parts[s][i]), the sum in fp32 in s order, rounded once to the grad
 * dtype.  parts [S, n] and grad [n] of `dtype` (bf16 / f32), 16-B aligned, n a
 * multiple of 8 (bf16) / 4 (f32).  Replaces the AccumulateGrad of the
 * reference's weight gradients (one GEMM per weight). */
int swh_dw_reduce(const void *parts, int32_t S, int64_t n, void *grad, int32_t dtype, void *stream);
/* Narrow-projection GEMM of the training forward / input gradient (the qkv and
 * o projections the reference runs as nn.Linear inside transformers' Qwen2
 * attention, through grpo_trainer.py:1793-1810 _get_per_token_logps_and_entropies
 * and its backward): C[M, N] = A[M, K] B[N, K]^T (+ bias[N]), bf16 in and out,
 * fp32 accumulation in a fixed K order.  N % 128 == 0, K % 64 == 0, leading
 * dimensions multiples of 8 elements, pointers 16-B aligned; else SWH_E_ARG. */
int swh_gemm_nt(const void *A, const void *B, const void *bias, void *C, int64_t M, int64_t N, int64_t K,
                int64_t lda, int64_t ldb, int64_t ldc, void *stream);
/* The same product for the wide projections (gate/up forward, the lm head of the
 * log-prob pass, the down input gradient against a transposed weight copy):
 * 256 x 256 tiles, one workgroup per CU, an eight-phase K loop (csrc/tgemm256.hip).
 * bf16 in and out, fp32 accumulation in ascending K (16-k MFMA steps), so a row's
 * result does not depend on its tile.  N % 8 == 0, K % 64 == 0, lda / ldb
 * multiples of 8 and ldc of 4 elements, A / B 16-B and C / bias 8-B aligned,
 * M * lda and N * ldb < 2^32; else SWH_E_ARG. */
int swh_gemm_nt256(const void *A, const void *B, const void *bias, void *C, int64_t M, int64_t N, int64_t K,
                   int64_t lda, int64_t ldb, int64_t ldc, void *stream);
/* Their weight gradient dW[N, K] += dY[M, N]^T X[M, K] (the AccumulateGrad of
 * the same nn.Linear weights), in two launches: swh_gemm_tn_partials writes
 * part[s][N][K] (fp32) = the sum over split s's tokens (S ranges of whole
 * 64-token steps, fp32 accumulation in token order), swh_gemm_tn_fold adds the S
 * partials in split order to grad (bf16 / f32, n = N K elements) and rounds
 * once.  colsum (nullable, [S][N] fp32): also the split's token sums of dY, the
 * bias gradient of the same nn.Linear (replaces a swh_colsum_partials pass over
 * dY), to be folded by swh_rmsnorm_dw_accum.  M % 64 == 0, N % 128 == 0,
 * K % 128 == 0, leading dimensions multiples of 8 elements, 16-B aligned
 * pointers; else SWH_E_ARG. */
int swh_gemm_tn_partials(const void *dY, const void *X, float *part, float *colsum, int64_t M, int64_t N, int64_t K,
                         int64_t lddy, int64_t ldx, int32_t S, void *stream);
int swh_gemm_tn_fold(const float *part, int32_t S, int64_t n, void *grad, int32_t dtype, void *stream);
/* The weight gradient on the swh_gemm_nt256 schedule (csrc/tgemm256.hip): part[s][N][K]
 * (fp32) = dY[tokens of split s]^T X, 256 x 256 tiles of (N, K), the tokens read
 * through ds_read_b64_tr_b16; S ranges of whole 64-token steps, each summed in
 * ascending token order; folded into the gradient by swh_gemm_tn_fold.  M % 64 == 0,
 * N and K % 16 == 0, leading dimensions multiples of 8 elements, pointers 16-B
 * aligned, M * ld * 2 < 2^31 bytes per operand; else SWH_E_ARG. */
int swh_gemm_tn256_partials(const void *dY, const void *X, float *part, int64_t M, int64_t N, int64_t K, int64_t lddy,
                            int64_t ldx, int32_t S, void *stream);
/* dst_f32[i] += src[i] (bf16/f32) — accumulate micro-batch grads in fp32. */
int swh_accumulate(float *dst, const void *src, int dtype, int64_t N, float scale, void *stream);

/* ---- a4: decoder kernels of the rollout engine -----------------------------
 * The transformer the reference runs through transformers' Qwen2/Llama
 * modeling code (third-party); GEMMs stay on hipBLASLt (MFMA), everything
 * between GEMMs is here.  bf16 in/out, fp32 math, rounding points as the
 * transformers bf16 modules (RMSNorm casts before the weight multiply).
 * The full-sequence kernels below that take `dtype` also run an fp32 model
 * (dtype SWH_F32: every tensor argument f32, no intermediate rounding — the
 * transformers fp32 modules); the decode kernels are bf16 only.            */
/* y = bf16(w * bf16(s * rsqrt(mean(s^2) + eps))), s = x (+ residual), the sum
 * s also written to residual_out when residual is given; rstd f32 [rows]
 * nullable (saved for the backward). */
int swh_rmsnorm_fwd(const void *x, const void *residual, void *residual_out, const void *weight,
                    int64_t rows, int64_t H, float eps, void *y, float *rstd, int32_t dtype, void *stream);
/* Backward: dx = rstd*(w*dy - n*mean(w*dy*n)), n = x*rstd; dw partial sums
 * f32 [ceil(rows/rows_per_block) x H] reduced by the caller. */
int swh_rmsnorm_bwd(const void *x, const void *weight, const float *rstd, const void *dy, int64_t rows, int64_t H,
                    void *dx, float *dw_partial, int64_t rows_per_block, const void *dres, int32_t dtype,
                    void *stream);
/* dres (nullable, bf16 [rows, H]): the gradient arriving through the residual
 * branch; dx = bf16(bf16(norm backward) + dres), the sum autograd forms where
 * the residual stream forks into the next RMSNorm.  swh_rmsnorm_dw_accum folds
 * the partial weight-gradient column sums into the bf16 gradient view:
 * grad_w = bf16(grad_w + bf16(sum over blocks)) (f32: grad_w += sum), in a fixed
 * order; above 64 partial rows it sums ranges of 32 rows first and uses
 * dw_partial as scratch (each range's first row is overwritten). */
int swh_rmsnorm_dw_accum(const float *dw_partial, int64_t nblocks, int64_t H, void *grad_w, int32_t dtype,
                         void *stream);
/* Column sums of x [rows, cols] (`dtype` bf16/f32, cols % 8 (bf16) / 4 (f32) == 0)
 * into fp32 partial rows part [ceil(rows / rows_per_chunk), cols], fixed order
 * (no atomics); swh_rmsnorm_dw_accum then folds them into a gradient view.  The
 * bias gradient of the q/k/v projection (the autograd of transformers'
 * nn.Linear bias in the reference's training forward). */
int swh_colsum_partials(const void *x, int64_t rows, int64_t cols, int64_t rows_per_chunk, float *part,
                        int32_t dtype, void *stream);
/* out[r, i] = bf16(bf16(silu(gu[r, i])) * gu[r, I + i]) — gate/up packed. */
int swh_silu_mul_fwd(const void *gu, int64_t rows, int64_t I, void *out, int32_t dtype, void *stream);
int swh_silu_mul_bwd(const void *gu, const void *dout, int64_t rows, int64_t I, void *dgu, int32_t dtype,
                     void *stream);
/* QKV split + rotate-half RoPE of the full-sequence forward (transformers
 * apply_rotary_pos_emb in bf16, with bf16-rounded cos/sin; the reference's
 * training / scoring forward, grpo_trainer.py:1249):
 *   forward  (backward = 0): qkv [B*L, (Hq+2Hkv) D] -> q [B,Hq,L,D],
 *            k [B,Hkv,L,D] rotated at positions[b*L + l], v [B,Hkv,L,D] copied;
 *   backward (backward = 1): q/k/v hold dq/dk/dv, qkv receives d qkv (the
 *            autograd of the bf16 ops: dx1 = bf16(bf16(dy1 c) + bf16(dy2 s)),
 *            dx2 = bf16(bf16(dy2 c) - bf16(dy1 s))).  D % 16 == 0. */
int swh_qkv_rope(void *qkv, const int64_t *positions, const float *rope_cos, const float *rope_sin, int64_t B,
                 int64_t L, int32_t Hq, int32_t Hkv, int32_t D, void *q, void *k, void *v, int32_t backward,
                 int32_t dtype, void *stream);
/* Causal GQA attention over full sequences (training / scoring / prefill),
 * bf16 [B, H, L, D] tensors (D = 64 or 128), fp32 softmax statistics.
 * Forward writes out and lse [B, Hq, L] (natural log of the row sum of
 * exp(scale * q k), the backward's statistic).  Backward takes dout and
 * writes dq, dk, dv (dk/dv summed over the Hq/Hkv query heads of each KV
 * head); delta [B, Hq, L] fp32 is workspace.  key_mask int32 [B, L] (0 = pad)
 * and first_valid int32 [B] are both null (pure causal) or both given: key k
 * is seen by query q iff k <= q and (key_mask[k] or (k == q and
 * q < first_valid)).  Replaces torch SDPA in the transformers Qwen2/Llama
 * attention of the reference's scoring and training forwards
 * (grpo_trainer.py:1249, ppo_trainer.py:86-96). */
int swh_attn_fwd(const void *q, const void *k, const void *v, int64_t B, int32_t Hq, int32_t Hkv, int64_t L,
                 int32_t D, float scale, const int32_t *key_mask, const int32_t *first_valid, void *out, float *lse,
                 void *stream);
int swh_attn_bwd(const void *q, const void *k, const void *v, const void *out, const void *dout, const float *lse,
                 int64_t B, int32_t Hq, int32_t Hkv, int64_t L, int32_t D, float scale, const int32_t *key_mask,
                 const int32_t *first_valid, float *delta, void *dq, void *dk, void *dv, void *stream);
/* swh_attn_bwd in parts, for callers that overlap them on two streams: bit 1
 * delta = rowsum(dO * O) (the other two read it), bit 2 dQ, bit 4 dK/dV.  dQ and
 * dK/dV are independent once delta is written.  parts = 7 is swh_attn_bwd. */
enum { SWH_ATTN_BWD_DELTA = 1, SWH_ATTN_BWD_DQ = 2, SWH_ATTN_BWD_DKDV = 4 };
int swh_attn_bwd_parts(const void *q, const void *k, const void *v, const void *out, const void *dout,
                       const float *lse, int64_t B, int32_t Hq, int32_t Hkv, int64_t L, int32_t D, float scale,
                       const int32_t *key_mask, const int32_t *first_valid, float *delta, void *dq, void *dk,
                       void *dv, int32_t parts, void *stream);
/* The same attention over operands given as views: an operand indexed
 * [B, H, L, D] (D contiguous, 16-B aligned) whose rows l < P live in segment 0
 * at sequence index b / div[0] and rows l >= P in segment 1 at b / div[1], each
 * with its own element strides per sequence, head and row (P = 0: segment 1
 * only).  G > 0: queries l < P of sequences b % G != 0 are neither computed nor
 * written (their output, lse and gradients do not exist; they contribute to no
 * dK / dV).  This is the GRPO shared-prompt forward (engine/model.py
 * hidden_states_grouped): Q/K/V of a group's prompt once per group (div G),
 * each row's completion (div 1), the output token-major [prompt tokens of the
 * groups | completion tokens of the rows, Hq D] for o_proj, dK / dV of the
 * prompt keys per row (div 1, summed over the group by the caller).
 * swh_attn_fwd / swh_attn_bwd_parts are these over plain [B, H, L, D] views. */
typedef struct swh_attn_view {
    void *base[2];
    int64_t sb[2], sh[2], sl[2]; /* element strides: per sequence (index b / div), per head, per row */
    int32_t div[2];
} swh_attn_view;
int swh_attn_fwd_v(const swh_attn_view *q, const swh_attn_view *k, const swh_attn_view *v, const swh_attn_view *out,
                   int64_t B, int32_t Hq, int32_t Hkv, int64_t L, int64_t P, int32_t G, int32_t D, float scale,
                   const int32_t *key_mask, const int32_t *first_valid, float *lse, void *stream);
int swh_attn_bwd_v_parts(const swh_attn_view *q, const swh_attn_view *k, const swh_attn_view *v,
                         const swh_attn_view *out, const swh_attn_view *dout, const float *lse, int64_t B, int32_t Hq,
                         int32_t Hkv, int64_t L, int64_t P, int32_t G, int32_t D, float scale,
                         const int32_t *key_mask, const int32_t *first_valid, float *delta, const swh_attn_view *dq,
                         const swh_attn_view *dk, const swh_attn_view *dv, int32_t parts, void *stream);

/* Folded RMSNorm weights for the decode GEMMs in ONE launch: for every job j of
 * the device-resident table jobs[njobs] = {W [rows, cols] bf16, w [cols] bf16,
 * out [rows, cols] bf16, rows, cols, row0 (prefix sum of rows)},
 * out[n][k] = bf16(W[n][k] * w[k]); cols % 8 == 0, 16-B aligned rows.
 * total_rows = sum of rows, njobs <= 256.  Run once per generate(): the policy update changes
 * W and w (transformers applies w inside Qwen2RMSNorm every token). */
int swh_fold_norm(const void *jobs, int32_t njobs, int64_t total_rows, void *stream);

/* Embedding weight gradient, deterministic (no atomics): grad_table[id] +=
 * sum of dy rows whose token is id, rows visited in the order given by a STABLE
 * sort of the ids (sorted_ids int64 [N], order int64 [N] = the sort's
 * permutation; ids outside [0, V) are skipped), summed in fp32 and folded in
 * once: bf16: g = bf16(g + bf16(sum)), f32: g += sum.  dy [N, H] and
 * grad_table [V, H] of `dtype`; workspace f32 >= swh_embedding_bwd_workspace_bytes.
 * Replaces the embedding backward (torch index_add_ / embedding_dense_backward)
 * of the reference's training forward (grpo_trainer.py:1249). */
int64_t swh_embedding_bwd_workspace_bytes(int64_t N, int64_t H);
int swh_embedding_bwd(const int64_t *sorted_ids, const int64_t *order, const void *dy, int64_t N, int64_t H, int64_t V,
                      void *grad_table, int32_t dtype, float *workspace, void *stream);

/* x[b, :] = table[ids[b], :] (bf16 rows of width H, H % 16 == 0); ss_out f32
 * [B, H/16] nullable: per 16-column chunk sums of squares of each row (the
 * RMSNorm statistic swh_decode_gemm takes as ss_in). */
int swh_embed_gather(const void *table, const int64_t *ids, int64_t B, int64_t H, void *x, float *ss_out,
                     void *stream);
/* One decode step of attention for every sequence.  state = device int32[2]
 * {s, P}: s is the index of the token the sampler produces in this step (the
 * same counter swh_sample_step reads), so the attention input is token s-1:
 * RoPE on its q/k at position prompt_len[b] + s - 1, k/v appended at cache
 * slot P + s - 1, softmax(q k^T * scale) v over slots
 * [P - prompt_len[b], P + s - 1].  Device-resident state lets one captured
 * graph serve every step and every prompt width.  A slot outside the cache
 * writes NaN outputs and leaves the cache untouched.
 * qkv bf16 [B, (Hq + 2 Hkv) D] (bias included); caches bf16 [B, Hkv, Tmax, D];
 * rope f32 [max_pos, D/2] cos and sin (already rounded to bf16 values);
 * out bf16 [B, Hq D]. */
int swh_attn_decode(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                    const float *rope_sin, const int32_t *prompt_len, const int32_t *state, int64_t B, int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax, float scale, void *out,
                    void *stream);
/* swh_attn_decode where the prompt keys / values of row b (cache slots
 * P - prompt_len[b] .. P - 1) are read from row prompt_row[b]'s cache: the G
 * generations of a GRPO prompt (RepeatSampler copies, trl/trainer/grpo_trainer.py:1096-1130)
 * hold identical prompt K/V, so one copy serves the group (HBM reads it once).
 * prompt_row int32 [B] (rows of one group: equal prompts and prompt_len); NULL
 * is the own row.  Generated keys and the appended slot stay per row. */
int swh_attn_decode_shared(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                           const float *rope_sin, const int32_t *prompt_len, const int32_t *prompt_row,
                           const int32_t *state, int64_t B, int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax,
                           float scale, void *out, void *stream);
/* swh_attn_decode_shared; out_frag = 1 writes `out` in the fragment order that
 * swh_decode_gemm_fragw reads with act_frag bit 1 (element (b, c) of [B, Hq*D] at
 * (((b/16) (Hq*D/32) + c/32) 64 + 16 ((c/8) % 4) + b % 16) 8 + c % 8), so o_proj
 * takes its A operand as contiguous 1 KB runs.  Same values as out_frag = 0.
 * out_frag = 1 needs B % 16 == 0, (Hq*D) % 32 == 0 and `out` 16-B aligned. */
int swh_attn_decode_shared_frag(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                                const float *rope_sin, const int32_t *prompt_len, const int32_t *prompt_row,
                                const int32_t *state, int64_t B, int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax,
                                float scale, void *out, int32_t out_frag, void *stream);

/* Weight-streaming decode GEMM Y[M,N] = X[M,K] W[N,K]^T (bf16, fp32 MFMA
 * accumulation, K % 64 == 0, 16-B aligned operands, ldy % 8 == 0) with the
 * decoder's neighbours fused:
 *   norm_w != NULL : X is replaced by RMSNorm(X) * norm_w (eps) in the prologue;
 *                    ss_in f32 [M, K/16] (nullable) = the producer's per
 *                    16-column chunk sums of squares of X (else computed here)
 *   bias   != NULL : + bias[N]
 *   residual != NULL: residual[M,N] = bf16(residual + bf16(XW^T)) in place
 *                     (row stride ldy; y unused); ss_out f32 [M, N/16]
 *                     (nullable) receives the new rows' chunk sums of squares
 *   silu != 0      : W has 2N rows (gate then up); y = bf16(bf16(silu(g)) * u)
 * Replaces the transformers q/k/v, o, gate/up, down and lm-head projections of
 * one decode step (plus their RMSNorm / SiLU / residual neighbours).
 * Small-N shapes split K over workgroups; the workspace (>=
 * swh_decode_gemm_workspace_bytes, ZEROED once at allocation, self-resetting
 * afterwards) holds the split counters and fp32 partial slabs. */
int64_t swh_decode_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K);
int swh_decode_gemm(const void *x, const void *w, int64_t M, int64_t N, int64_t K, const void *norm_w, float eps,
                    const void *bias, void *residual, int32_t silu, void *y, int64_t ldy, const float *ss_in,
                    float *ss_out, void *workspace, int64_t workspace_bytes, void *stream);

/* Bandwidth-regime decode GEMM over a PACKED weight (Llama-3-8B decode at 64
 * rows; replaces the same reference call sites as swh_decode_gemm — the policy
 * forward inside unwrapped_model.generate(), trl/trainer/grpo_trainer.py:1114-1130).
 * swh_wide_pack writes W (or the folded-norm weight bf16(W * norm_w)) in the
 * MFMA-fragment order: each 16-row group's 128-k rounds are contiguous 4 KB
 * runs.  swh_wide_gemm_packed then computes what swh_decode_gemm computes on
 * the row-major weight with norm_w == NULL (bit-identical), for shapes
 * swh_wide_gemm_eligible accepts (M <= 64, K % 128 == 0, N (2N with silu)
 * % 128 == 0 and >= 1024); anything else is SWH_E_ARG. */
int swh_wide_gemm_eligible(int64_t M, int64_t N, int64_t K, int32_t silu);
int swh_wide_pack(const void *w, const void *norm_w, int64_t N, int64_t K, int32_t silu, void *dst, void *stream);
int swh_wide_gemm_packed(const void *x, const void *w, int64_t M, int64_t N, int64_t K, float eps, const void *bias,
                         void *residual, int32_t silu, void *y, int64_t ldy, const float *ss_in, float *ss_out,
                         void *workspace, int64_t workspace_bytes, void *stream);

/* swh_decode_gemm over a weight in the MFMA-fragment order (the Qwen2.5-0.5B
 * decode projections: qkv, o, gate/up, down; same reference call sites as
 * swh_decode_gemm, trl/trainer/grpo_trainer.py:1114-1130): swh_frag_pack
 * writes W [N, K] ([2N, K] gate|up with silu; K % 128 == 0), or the folded-norm
 * weight bf16(W * norm_w), in swh_wide_pack's order for any 16-row group
 * count — per 16-row group (8 gate + 8 up rows with silu) and 32-wide k-step,
 * the 64 lanes' 16-B fragments contiguous — so each weight load of a wave is
 * one 1 KB run instead of 16 rows x 64 B.  swh_decode_gemm_fragw then computes
 * what swh_decode_gemm computes on the row-major W with norm_w == NULL
 * (bit-identical): residual, bias, SiLU-gate and folded-norm row scale (ss_in)
 * epilogues.  act_frag (M % 16 == 0): bit 0 — the SiLU output y is written in
 * the same fragment order over its [M, N] (N % 32 == 0; 16-row groups), bit 1 —
 * X (a residual projection's input, e.g. that SiLU output) is read in it: the
 * decode gate/up -> down hand-off without row-major activations.  A shape whose
 * kernels cannot honour a requested bit is SWH_E_ARG (no fallback). */
int swh_frag_pack(const void *w, const void *norm_w, int64_t N, int64_t K, int32_t silu, void *dst, void *stream);
int swh_decode_gemm_fragw(const void *x, const void *w, int64_t M, int64_t N, int64_t K, float eps, const void *bias,
                          void *residual, int32_t silu, void *y, int64_t ldy, const float *ss_in, float *ss_out,
                          int32_t act_frag, void *workspace, int64_t workspace_bytes, void *stream);

/* Decode lm head with the sampler fused into its epilogue: RMSNorm(X) W^T
 * (as swh_decode_gemm with norm_w / ss_in) and, per row, the token that
 * swh_sample_step would draw from those logits with the same rng / step
 * (Gumbel-max over bf16 logits, EOS suppression, temperature, greedy) —
 * without materialising the [M, V] logits.  Bookkeeping (finished, pad, EOS,
 * out_tokens[:, *step], cur_tokens) as swh_sample_step.  Unfiltered sampling
 * only: top-k / top-p / min-p / repetition penalty return SWH_E_ARG (use the
 * logits + swh_sample_step path).  K % 64 == 0, K <= 1024, V % 16 == 0.
 * Replaces the reference's per-step lm_head + LogitsProcessorList +
 * torch.multinomial of transformers `_sample` (grpo_trainer.py:1804). */
int64_t swh_lm_head_sample_workspace_bytes(int64_t M, int64_t V, int64_t K);
int swh_lm_head_sample(const void *x, const void *w, int64_t M, int64_t V, int64_t K, const void *norm_w, float eps,
                       const float *ss_in, const swh_sample_params *params, const uint64_t *rng, const int32_t *step,
                       int32_t *finished, int64_t *out_tokens, int64_t out_ld, int64_t *cur_tokens, void *workspace,
                       int64_t workspace_bytes, void *stream);

/* swh_lm_head_sample plus the next decode step's input in the same launches:
 * x_next[b] = embed[token drawn for row b] and ss_next its RMSNorm partial
 * sums (as swh_embed_gather), and *step advanced by one once every row has
 * read it (as swh_step_advance).  One replayable decode step ends here; the
 * workspace (>= swh_lm_head_sample_workspace_bytes) must be ZEROED once at
 * allocation (a self-resetting ticket lives at its end).  Replaces the
 * per-token `input_ids = cat(input_ids, next_tokens)` / embedding lookup /
 * cache_position advance of transformers `_sample` (grpo_trainer.py:1804). */
int swh_lm_head_sample_step(const void *x, const void *w, int64_t M, int64_t V, int64_t K, const void *norm_w,
                            float eps, const float *ss_in, const swh_sample_params *params, const uint64_t *rng,
                            int32_t *step, int32_t *finished, int64_t *out_tokens, int64_t out_ld,
                            int64_t *cur_tokens, const void *embed, void *x_next, float *ss_next, void *workspace,
                            int64_t workspace_bytes, void *stream);
/* The two entries above over the folded lm-head weight packed by swh_frag_pack
 * (norm_w NULL: the row scale comes from ss_in; K % 128 == 0): same draws.
 * K > 1024 (Llama-3-8B): the same order as swh_wide_pack writes, through the
 * bandwidth-regime GEMM's 256-row tiles with the sampler as their epilogue, for
 * M <= 64 and V % 256 == 0 (else SWH_E_ARG: logits + swh_sample_step); the
 * draws equal swh_sample_step over the logits those tiles write. */
int swh_lm_head_sample_fragw(const void *x, const void *w, int64_t M, int64_t V, int64_t K, float eps,
                             const float *ss_in, const swh_sample_params *params, const uint64_t *rng,
                             const int32_t *step, int32_t *finished, int64_t *out_tokens, int64_t out_ld,
                             int64_t *cur_tokens, void *workspace, int64_t workspace_bytes, void *stream);
int swh_lm_head_sample_step_fragw(const void *x, const void *w, int64_t M, int64_t V, int64_t K, float eps,
                                  const float *ss_in, const swh_sample_params *params, const uint64_t *rng,
                                  int32_t *step, int32_t *finished, int64_t *out_tokens, int64_t out_ld,
                                  int64_t *cur_tokens, const void *embed, void *x_next, float *ss_next,
                                  void *workspace, int64_t workspace_bytes, void *stream);

/* The fused lm-head sampler that also writes the drawn token's log-prob under the
 * processed distribution, out_logp[b * out_ld + *step] = z - logsumexp(z) over the
 * row's processed scores z (logits / T with EOS suppression; greedy: the logits),
 * as swh_sample_step's out_logp does over materialised logits: each tile also
 * folds a per-row (max, sum e^(z - max)), merged in the finalize; the drawn
 * score is recovered from its Gumbel key (within one fp32 rounding).  Same draws
 * as swh_lm_head_sample.  frag_weights 0: W row-major ([V, K], norm_w or ss_in
 * as swh_lm_head_sample), 1: the frag_pack order (norm_w NULL, ss_in).  embed
 * NULL: no next-step input and *step is not advanced (swh_lm_head_sample);
 * otherwise as swh_lm_head_sample_step.  K <= 1024 (the tile kernel) only: K >
 * 1024 is SWH_E_ARG (logits + swh_sample_step).  Replaces the rollout log-probs
 * PPO computes from the generation's scores (trl/trainer/utils.py:1092-1094
 * output_scores, ppo_trainer.py:440 selective_log_softmax of logits / (T + 1e-7))
 * with no extra pass over the logits. */
int swh_lm_head_sample_logp(const void *x, const void *w, int64_t M, int64_t V, int64_t K, const void *norm_w,
                            float eps, const float *ss_in, int32_t frag_weights, const swh_sample_params *params,
                            const uint64_t *rng, int32_t *step, int32_t *finished, int64_t *out_tokens, int64_t out_ld,
                            int64_t *cur_tokens, float *out_logp, const void *embed, void *x_next, float *ss_next,
                            void *workspace, int64_t workspace_bytes, void *stream);

/* swh_attn_decode_shared_frag whose launch also carries >= l3_wgs Infinity Cache
 * warm-up workgroups (rounded up to whole grid rows of Hkv) on the CUs the
 * attention's B x Hkv workgroups leave idle: they read the l3_njobs (<= 8)
 * ranges {const void *ptr, int64_t bytes / 16, int64_t 0} (16-B aligned device
 * memory) in contiguous shares and discard the data, so the projections that
 * follow (o_proj and down_proj of this layer, qkv of the next) find their
 * weights on-die; l3_sink >= rounded workgroups x 512 uint32 of
 * scratch.  Results identical to swh_attn_decode_shared_frag. */
int swh_attn_decode_l3(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos, const float *rope_sin,
                       const int32_t *prompt_len, const int32_t *prompt_row, const int32_t *state, int64_t B,
                       int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax, float scale, void *out, int32_t out_frag,
                       const void *l3_jobs, int32_t l3_njobs, int32_t l3_wgs, void *l3_sink, void *stream);

/* ---- GPT-2 family (BASELINE.json config 1) --------------------------------
 * transformers GPT2Block's LayerNorms and NewGELUActivation (the modeling code
 * the reference's tiny-random-GPT2 tests run through grpo_trainer.py:1249 /
 * :1804), bf16 or fp32.  dtype SWH_BF16 / SWH_F32; every tensor in it.
 *
 * swh_layernorm_fwd: s = residual ? dtype(x + residual) : x (written to s_out
 * when residual is given), y = dtype((s - mean) * rstd * w + b) with fp32
 * mean, biased variance and rstd = 1/sqrt(var + eps) per row (saved). */
int swh_layernorm_fwd(const void *x, const void *residual, const void *w, const void *b, int64_t rows, int64_t H,
                      float eps, void *y, void *s_out, float *mean, float *rstd, int32_t dtype, void *stream);
/* Rows of partial sums the backward writes: ceil(rows / rows_per_block). */
int64_t swh_layernorm_bwd_partial_rows(int64_t rows, int64_t rows_per_block);
/* dx = rstd (g - mean(g) - xhat mean(g xhat)) + dres (nullable), g = dy w;
 * part_w / part_b (nullable together) [partial_rows][H] fp32: per block of
 * rows_per_block rows, sum dy * xhat and sum dy in fixed row order
 * (fold them into the gradient views with swh_rmsnorm_dw_accum). */
int swh_layernorm_bwd(const void *s, const void *w, const float *mean, const float *rstd, const void *dy,
                      const void *dres, int64_t rows, int64_t H, int64_t rows_per_block, void *dx, float *part_w,
                      float *part_b, int32_t dtype, void *stream);
/* gelu_new: y = 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))) over n
 * elements, rounded to dtype after each torch op of the reference activation
 * (exact fp32 for SWH_F32); the backward is the analytic derivative in fp32. */
int swh_gelu_tanh_fwd(const void *x, int64_t n, void *y, int32_t dtype, void *stream);
int swh_gelu_tanh_bwd(const void *x, const void *dy, int64_t n, void *dx, int32_t dtype, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SWH_TRL_AMD_H */
