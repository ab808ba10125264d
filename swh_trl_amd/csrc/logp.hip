// Fused temperature-scaled log-softmax gather + entropy (+ its backward).
//
// Replaces trl/trainer/utils.py:1430-1462 (selective_log_softmax) and
// :1465-1490 (entropy_from_logits) together with the `logits / temperature`
// of grpo_trainer.py:1254 and ppo_trainer.py:446,558.
//
// HBM-bound: one 16-byte coalesced load per lane per step, single pass over
// each row keeping an online (max, sum e^{z-m}, sum e^{z-m}(z-m)) triple in
// registers; wave shuffles + one LDS round merge the 4 waves.  Algorithmic
// bytes per row: V * sizeof(logit) read (fwd); 2 * V * sizeof(logit) (bwd).
#include "common.hpp"

namespace swh {
namespace {

constexpr int kThreads = 256;

struct RowAddr {
    int64_t outer, inner, s_outer, s_inner;
    __device__ __forceinline__ int64_t off(int64_t r) const {
        const int64_t o = r / inner, i = r - o * inner;
        return o * s_outer + i * s_inner;
    }
};

// z = x / T with a true division (the reference divides, it does not multiply
// by 1/T); optionally rounded back to the logits dtype like a bf16 tensor op.
template <int DT>
__device__ __forceinline__ float scaled(float x, float inv_t, float t, bool has_t, bool round_scaled) {
    (void)inv_t;
    if (!has_t) return x;
    const float z = x / t;
    return round_scaled ? Elem<DT>::round(z) : z;
}

template <int DT>
__global__ __launch_bounds__(kThreads) void logp_entropy_fwd_kernel(
    const typename Elem<DT>::T *__restrict__ logits, RowAddr ra, int64_t V, const int64_t *__restrict__ ids,
    float t, int flags, float *__restrict__ logp, float *__restrict__ entropy, float *__restrict__ lse) {
    using T = typename Elem<DT>::T;
    constexpr int PV = kPerVec<DT>;
    __shared__ float red[3 * (kThreads / kWave)];
    const int64_t r = blockIdx.x;
    const T *row = logits + ra.off(r);
    const bool has_t = (t != 1.0f);
    const bool rs = (flags & SWH_LOGP_ROUND_SCALED) != 0;
    const float inv_t = 1.0f / t;

    // Head elements until 16-byte alignment, vector body, tail.
    const uintptr_t addr = reinterpret_cast<uintptr_t>(row);
    int64_t head = (int64_t)(((16 - (addr & 15)) & 15) / sizeof(T));
    if (head > V) head = V;
    const int64_t nvec = (V - head) / PV;
    const int64_t body_end = head + nvec * PV;

    SoftState st = soft_init();
    for (int64_t j = threadIdx.x; j < head; j += kThreads) {
        float z = scaled<DT>(Elem<DT>::load(row + j), inv_t, t, has_t, rs);
        soft_fold<1>(st, &z);
    }
    const uint4 *vrow = reinterpret_cast<const uint4 *>(row + head);
    int64_t v = threadIdx.x;
    for (; v + kThreads < nvec; v += 2 * kThreads) {
        const uint4 a = ld_nt(vrow + v);
        const uint4 b = ld_nt(vrow + v + kThreads);
        float za[PV], zb[PV];
        unpack16<DT>(a, za);
        unpack16<DT>(b, zb);
#pragma unroll
        for (int k = 0; k < PV; ++k) {
            za[k] = scaled<DT>(za[k], inv_t, t, has_t, rs);
            zb[k] = scaled<DT>(zb[k], inv_t, t, has_t, rs);
        }
        soft_fold<PV>(st, za);
        soft_fold<PV>(st, zb);
    }
    for (; v < nvec; v += kThreads) {
        float za[PV];
        unpack16<DT>(ld_nt(vrow + v), za);
#pragma unroll
        for (int k = 0; k < PV; ++k) za[k] = scaled<DT>(za[k], inv_t, t, has_t, rs);
        soft_fold<PV>(st, za);
    }
    for (int64_t j = body_end + threadIdx.x; j < V; j += kThreads) {
        float z = scaled<DT>(Elem<DT>::load(row + j), inv_t, t, has_t, rs);
        soft_fold<1>(st, &z);
    }
    st = block_soft(st, red);
    if (threadIdx.x == 0) {
        const float ls1 = fast_log(st.s1);
        if (lse) lse[r] = st.m + ls1;
        if (entropy) entropy[r] = ls1 - st.s2 / st.s1;
        if (logp) {
            const int64_t id = ids[r];
            float out = __builtin_nanf("");
            if (id >= 0 && id < V) {
                const float zid = scaled<DT>(Elem<DT>::load(row + id), inv_t, t, has_t, rs);
                out = (zid - st.m) - ls1;  // same association as the log_softmax epilogue
            }
            logp[r] = out;
        }
    }
}

#ifndef SWH_LOGP_BWD_U
#define SWH_LOGP_BWD_U 4
#endif
template <int DT>
__global__ __launch_bounds__(kThreads) void logp_bwd_kernel(
    const typename Elem<DT>::T *__restrict__ logits, RowAddr ra, int64_t V, const int64_t *__restrict__ ids,
    float t, int flags, const float *__restrict__ lse, const float *__restrict__ dlogp,
    typename Elem<DT>::T *__restrict__ dlogits, RowAddr rd) {
    using T = typename Elem<DT>::T;
    constexpr int PV = kPerVec<DT>;
    const int64_t r = blockIdx.x;
    const T *row = logits + ra.off(r);
    T *drow = dlogits + rd.off(r);
    const bool has_t = (t != 1.0f);
    const bool rs = (flags & SWH_LOGP_ROUND_SCALED) != 0;
    const float inv_t = 1.0f / t;
    const float L = lse[r];
    const float g = dlogp[r] * inv_t;
    const int64_t id = ids[r];

    auto grad = [&](float x, int64_t j) -> float {
        const float z = scaled<DT>(x, inv_t, t, has_t, rs);
        const float p = fast_exp(z - L);
        return g * ((j == id ? 1.f : 0.f) - p);
    };
    auto store = [&](int64_t j, float v) {
        if constexpr (DT == SWH_F32) drow[j] = v;
        else if constexpr (DT == SWH_BF16) drow[j] = f32_to_bf16_bits(v);
        else drow[j] = f32_to_f16_bits(v);
    };

    const uintptr_t a_in = reinterpret_cast<uintptr_t>(row), a_out = reinterpret_cast<uintptr_t>(drow);
    const bool vec_ok = ((a_in & 15) == (a_out & 15));
    int64_t head = vec_ok ? (int64_t)(((16 - (a_in & 15)) & 15) / sizeof(T)) : V;
    if (head > V) head = V;
    const int64_t nvec = (V - head) / PV;
    const int64_t body_end = head + nvec * PV;
    for (int64_t j = threadIdx.x; j < head; j += kThreads) store(j, grad(Elem<DT>::load(row + j), j));
    const uint4 *vin = reinterpret_cast<const uint4 *>(row + head);
    uint4 *vout = reinterpret_cast<uint4 *>(drow + head);
    // SWH_LOGP_BWD_U vectors per thread and trip, every load issued before the math
    constexpr int U = SWH_LOGP_BWD_U;
    int64_t v = threadIdx.x;
    for (; v + (U - 1) * kThreads < nvec; v += U * kThreads) {
        uint4 in[U];
#pragma unroll
        for (int u = 0; u < U; ++u) in[u] = ld_nt(vin + v + u * kThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float x[PV];
            unpack16<DT>(in[u], x);
            const int64_t j0 = head + (v + u * kThreads) * PV;
            uint32_t w[4];
            if constexpr (DT == SWH_F32) {
#pragma unroll
                for (int k = 0; k < 4; ++k) w[k] = __float_as_uint(grad(x[k], j0 + k));
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float lo = grad(x[2 * k], j0 + 2 * k), hi = grad(x[2 * k + 1], j0 + 2 * k + 1);
                    const uint32_t blo = (DT == SWH_BF16) ? f32_to_bf16_bits(lo) : f32_to_f16_bits(lo);
                    const uint32_t bhi = (DT == SWH_BF16) ? f32_to_bf16_bits(hi) : f32_to_f16_bits(hi);
                    w[k] = blo | (bhi << 16);
                }
            }
            st_nt(vout + v + u * kThreads, uint4{w[0], w[1], w[2], w[3]});
        }
    }
    for (; v < nvec; v += kThreads) {
        float x[PV];
        unpack16<DT>(ld_nt(vin + v), x);
        const int64_t j0 = head + v * PV;
        uint32_t w[4];
        if constexpr (DT == SWH_F32) {
#pragma unroll
            for (int k = 0; k < 4; ++k) w[k] = __float_as_uint(grad(x[k], j0 + k));
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float lo = grad(x[2 * k], j0 + 2 * k), hi = grad(x[2 * k + 1], j0 + 2 * k + 1);
                const uint32_t blo = (DT == SWH_BF16) ? f32_to_bf16_bits(lo) : f32_to_f16_bits(lo);
                const uint32_t bhi = (DT == SWH_BF16) ? f32_to_bf16_bits(hi) : f32_to_f16_bits(hi);
                w[k] = blo | (bhi << 16);
            }
        }
        st_nt(vout + v, uint4{w[0], w[1], w[2], w[3]});
    }
    for (int64_t j = body_end + threadIdx.x; j < V; j += kThreads) store(j, grad(Elem<DT>::load(row + j), j));
}

// Half-precision rows of V <= 1024: the reference's bf16/fp16 branch
// (utils.py:1451-1459) is `log_softmax(row)` then gather, and its own test
// (test_utils.py:540-558) asks for bit equality with torch's log_softmax.  For
// these widths torch's device kernel is the persistent warp softmax (ATen
// PersistentSoftmax.cuh, softmax_warp_forward): WS = min(2^ceil(log2 V), 64)
// lanes per row, lane l holds elements l + it*WS (it < 2^ceil(log2 V)/WS,
// -inf past V), a sequential per-lane max / sum of exp(x - max) in it order,
// then xor-butterfly merges (offsets WS/2 .. 1) with max(a, b) = a < b ? b : a
// and a + b; out = (x - max) - log(sum) in fp32, rounded once (RNE).  This
// kernel performs exactly those fp32 operations in that order, with the
// accurate expf / logf (not the fast forms the fused kernel uses), so the
// gathered value is the same bits.  One WS-lane group per row.
template <int DT>
__global__ __launch_bounds__(kThreads) void log_softmax_gather_exact_kernel(const uint16_t *__restrict__ logits,
                                                                           RowAddr ra, int V, int ws, int iters,
                                                                           const int64_t *__restrict__ ids,
                                                                           int64_t R, uint16_t *__restrict__ out) {
    const int lane = threadIdx.x & (ws - 1);
    const int64_t r = ((int64_t)blockIdx.x * kThreads + threadIdx.x) / ws;
    const bool live = r < R;  // dead groups still take part in the shuffles of their wave
    const uint16_t *row = logits + ra.off(live ? r : 0);
    float e[16];
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int j = lane + it * ws;
        e[it] = (it < iters && j < V) ? Elem<DT>::load(row + j) : kNegInf;
    }
    float mx = e[0];
#pragma unroll
    for (int it = 0; it < 16; ++it)
        if (it < iters) mx = mx > e[it] ? mx : e[it];
    for (int off = ws / 2; off > 0; off >>= 1) {
        const float b = __shfl_xor(mx, off, ws);
        mx = mx < b ? b : mx;
    }
    float sum = 0.f;
#pragma unroll
    for (int it = 0; it < 16; ++it)
        if (it < iters) sum += expf(e[it] - mx);
    for (int off = ws / 2; off > 0; off >>= 1) sum = sum + __shfl_xor(sum, off, ws);
    if (!live || lane != 0) return;
    const float ls = logf(sum);
    const int64_t id = ids[r];
    float v = __builtin_nanf("");
    if (id >= 0 && id < V) v = (Elem<DT>::load(row + id) - mx) - ls;
    out[r] = (DT == SWH_BF16) ? f32_to_bf16_bits(v) : f32_to_f16_bits(v);
}

bool rows_ok(int64_t outer, int64_t inner, int64_t V) {
    return outer >= 0 && inner >= 0 && V > 0 && outer * inner < (int64_t)1 << 31;
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int swh_logp_entropy_fwd(const void *logits, int dtype, int64_t rows_outer, int64_t rows_inner,
                                    int64_t stride_outer, int64_t stride_inner, int64_t V, const int64_t *ids,
                                    float temperature, int flags, float *logp, float *entropy, float *lse,
                                    void *stream) {
    if (!rows_ok(rows_outer, rows_inner, V) || !(temperature > 0.f)) return SWH_E_ARG;
    const int64_t R = rows_outer * rows_inner;
    if (R == 0) return SWH_OK;  // empty batch: nothing to read (buffers may be null)
    if (!logits || (logp && !ids)) return SWH_E_ARG;
    RowAddr ra{rows_outer, rows_inner, stride_outer, stride_inner};
    hipStream_t s = static_cast<hipStream_t>(stream);
    dim3 grid((unsigned)R), block(kThreads);
    switch (dtype) {
    case SWH_BF16:
        logp_entropy_fwd_kernel<SWH_BF16><<<grid, block, 0, s>>>(static_cast<const uint16_t *>(logits), ra, V, ids,
                                                                  temperature, flags, logp, entropy, lse);
        break;
    case SWH_F16:
        logp_entropy_fwd_kernel<SWH_F16><<<grid, block, 0, s>>>(static_cast<const uint16_t *>(logits), ra, V, ids,
                                                                 temperature, flags, logp, entropy, lse);
        break;
    case SWH_F32:
        logp_entropy_fwd_kernel<SWH_F32><<<grid, block, 0, s>>>(static_cast<const float *>(logits), ra, V, ids,
                                                                 temperature, flags, logp, entropy, lse);
        break;
    default:
        return SWH_E_DTYPE;
    }
    return launch_status();
}

extern "C" int swh_log_softmax_gather_exact(const void *logits, int dtype, int64_t rows_outer, int64_t rows_inner,
                                            int64_t stride_outer, int64_t stride_inner, int64_t V,
                                            const int64_t *ids, void *out, void *stream) {
    if (!rows_ok(rows_outer, rows_inner, V) || V > 1024) return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F16) return SWH_E_DTYPE;
    const int64_t R = rows_outer * rows_inner;
    if (R == 0) return SWH_OK;
    if (!logits || !ids || !out) return SWH_E_ARG;
    int p2 = 1;
    while (p2 < V) p2 <<= 1;
    const int ws = p2 < kWave ? p2 : kWave, iters = p2 / ws;
    RowAddr ra{rows_outer, rows_inner, stride_outer, stride_inner};
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t groups_per_block = kThreads / ws;
    dim3 grid((unsigned)((R + groups_per_block - 1) / groups_per_block)), block(kThreads);
    const uint16_t *lg = static_cast<const uint16_t *>(logits);
    uint16_t *o = static_cast<uint16_t *>(out);
    if (dtype == SWH_BF16)
        log_softmax_gather_exact_kernel<SWH_BF16><<<grid, block, 0, s>>>(lg, ra, (int)V, ws, iters, ids, R, o);
    else
        log_softmax_gather_exact_kernel<SWH_F16><<<grid, block, 0, s>>>(lg, ra, (int)V, ws, iters, ids, R, o);
    return launch_status();
}

extern "C" int swh_logp_bwd(const void *logits, int dtype, int64_t rows_outer, int64_t rows_inner,
                            int64_t stride_outer, int64_t stride_inner, int64_t V, const int64_t *ids,
                            float temperature, int flags, const float *lse, const float *dlogp, void *dlogits,
                            int64_t dstride_outer, int64_t dstride_inner, void *stream) {
    if (!rows_ok(rows_outer, rows_inner, V) || !(temperature > 0.f)) return SWH_E_ARG;
    const int64_t R = rows_outer * rows_inner;
    if (R == 0) return SWH_OK;  // empty batch (buffers may be null)
    if (!logits || !ids || !lse || !dlogp || !dlogits) return SWH_E_ARG;
    RowAddr ra{rows_outer, rows_inner, stride_outer, stride_inner};
    RowAddr rd{rows_outer, rows_inner, dstride_outer, dstride_inner};
    hipStream_t s = static_cast<hipStream_t>(stream);
    dim3 grid((unsigned)R), block(kThreads);
    switch (dtype) {
    case SWH_BF16:
        logp_bwd_kernel<SWH_BF16><<<grid, block, 0, s>>>(static_cast<const uint16_t *>(logits), ra, V, ids,
                                                          temperature, flags, lse, dlogp,
                                                          static_cast<uint16_t *>(dlogits), rd);
        break;
    case SWH_F16:
        logp_bwd_kernel<SWH_F16><<<grid, block, 0, s>>>(static_cast<const uint16_t *>(logits), ra, V, ids,
                                                         temperature, flags, lse, dlogp,
                                                         static_cast<uint16_t *>(dlogits), rd);
        break;
    case SWH_F32:
        logp_bwd_kernel<SWH_F32><<<grid, block, 0, s>>>(static_cast<const float *>(logits), ra, V, ids, temperature,
                                                         flags, lse, dlogp, static_cast<float *>(dlogits), rd);
        break;
    default:
        return SWH_E_DTYPE;
    }
    return launch_status();
}
