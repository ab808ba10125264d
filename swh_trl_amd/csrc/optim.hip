// Flat-buffer optimizer kernels: global grad-norm clip + decoupled AdamW.
//
// Replaces the optimizer the reference gets from transformers'
// Trainer.create_optimizer (torch.optim.AdamW) and the
// `clip_grad_norm_(max_grad_norm=1.0)` of the Trainer loop.  All parameters
// live in ONE flat buffer (the host lays every weight out as a view into it),
// so the whole update is one HBM-bound streaming kernel instead of a
// multi-tensor list, and the clip coefficient never leaves the device.
// Algorithmic bytes per parameter: grad 2 (bf16) + master 8 + m 8 + v 8 +
// model copy 2 = 28 B.
#include "common.hpp"

namespace swh {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxPartials = 1024;

template <int DT>
__global__ __launch_bounds__(kThreads) void sqnorm_kernel(const typename Elem<DT>::T *__restrict__ g, int64_t N,
                                                          float *__restrict__ partials) {
    __shared__ float red[kThreads / kWave];
    float acc[1] = {0.f};
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    row_foreach<DT, true>(g, (int64_t)0, N, (int)(blockIdx.x * kThreads + threadIdx.x), (int)stride,
                          [&](int64_t, float x) { acc[0] = fmaf(x, x, acc[0]); });
    block_sum<1>(acc, red);
    if (threadIdx.x == 0) partials[blockIdx.x] = acc[0];
}

__global__ __launch_bounds__(kThreads) void finalize_clip_kernel(const float *__restrict__ partials, int64_t n,
                                                                 float max_norm, float *__restrict__ out) {
    __shared__ double red[kThreads / kWave];
    double a[1] = {0.0};
    for (int64_t i = threadIdx.x; i < n; i += kThreads) a[0] += (double)partials[i];
    block_sum_d<1>(a, red);
    if (threadIdx.x == 0) {
        const float norm = (float)sqrt(a[0]);
        out[0] = norm;
        float coef = 1.f;
        if (max_norm > 0.f) coef = fminf(1.f, max_norm / (norm + 1e-6f));
        out[1] = coef;
    }
}

constexpr int kMaxNoDecay = 1024;  // no-decay ranges held in LDS

// WM: 0 = no model copy, SWH_BF16 = bf16 copy, SWH_F32 = fp32 copy.  NR: the
// no-decay range table is consulted (binary search in LDS per float4 group;
// ranges are 4-aligned so a group never straddles one).
template <int GDT, int WM, bool NR>
__global__ __launch_bounds__(kThreads) void adamw_kernel(float *__restrict__ p, float *__restrict__ m,
                                                         float *__restrict__ v,
                                                         const typename Elem<GDT>::T *__restrict__ g,
                                                         uint16_t *__restrict__ model,
                                                         float *__restrict__ model32, int64_t N, float lr,
                                                         float b1, float b2, float eps, float wd, float step_size,
                                                         float bc2_sqrt, const float *__restrict__ clip,
                                                         const int64_t *__restrict__ nd, int nnd) {
    __shared__ int64_t tab[NR ? 2 * kMaxNoDecay : 1];
    if constexpr (NR) {
        for (int i = threadIdx.x; i < 2 * nnd; i += kThreads) tab[i] = nd[i];
        __syncthreads();
    }
    const float cf = clip ? clip[1] : 1.f;
    const float decay_on = 1.f - lr * wd;
    // 1 - lr*wd, or 1 inside a no-decay range
    auto decay_at = [&](int64_t e) {
        if constexpr (!NR) {
            return decay_on;
        } else {
            int lo = 0, hi = nnd - 1, hit = -1;
            while (lo <= hi) {
                const int mid = (lo + hi) >> 1;
                if (tab[2 * mid] <= e) { hit = mid; lo = mid + 1; }
                else hi = mid - 1;
            }
            return (hit >= 0 && e < tab[2 * hit + 1]) ? 1.f : decay_on;
        }
    };
    const int64_t n4 = N / 4;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    auto upd = [&](float &pp, float &mm, float &vv, float gg, float decay) {
        gg *= cf;
        pp *= decay;
        mm = fmaf(1.f - b1, gg - mm, mm);       // exp_avg.lerp_(grad, 1 - beta1)
        vv = fmaf((1.f - b2) * gg, gg, vv * b2);  // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
        const float denom = sqrtf(vv) / bc2_sqrt + eps;
        pp = pp - step_size * (mm / denom);
    };
    // U grid-strided float4 groups per trip, every load of the trip issued before any math
    constexpr int U = 2;
    for (int64_t i0 = (int64_t)blockIdx.x * kThreads + threadIdx.x; i0 < n4; i0 += U * stride) {
        float4 pp[U], mm[U], vv[U];
        float gg[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i < n4) {
                pp[u] = reinterpret_cast<float4 *>(p)[i];
                mm[u] = reinterpret_cast<float4 *>(m)[i];
                vv[u] = reinterpret_cast<float4 *>(v)[i];
                if constexpr (GDT == SWH_F32) {
                    const float4 t = reinterpret_cast<const float4 *>(g)[i];
                    gg[u][0] = t.x; gg[u][1] = t.y; gg[u][2] = t.z; gg[u][3] = t.w;
                } else {
                    const uint2 t = reinterpret_cast<const uint2 *>(g)[i];
                    gg[u][0] = Elem<GDT>::load(reinterpret_cast<const uint16_t *>(&t.x));
                    gg[u][1] = Elem<GDT>::load(reinterpret_cast<const uint16_t *>(&t.x) + 1);
                    gg[u][2] = Elem<GDT>::load(reinterpret_cast<const uint16_t *>(&t.y));
                    gg[u][3] = Elem<GDT>::load(reinterpret_cast<const uint16_t *>(&t.y) + 1);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i >= n4) break;
            const float dc = decay_at(4 * i);
            upd(pp[u].x, mm[u].x, vv[u].x, gg[u][0], dc);
            upd(pp[u].y, mm[u].y, vv[u].y, gg[u][1], dc);
            upd(pp[u].z, mm[u].z, vv[u].z, gg[u][2], dc);
            upd(pp[u].w, mm[u].w, vv[u].w, gg[u][3], dc);
            reinterpret_cast<float4 *>(p)[i] = pp[u];
            reinterpret_cast<float4 *>(m)[i] = mm[u];
            reinterpret_cast<float4 *>(v)[i] = vv[u];
            if constexpr (WM == SWH_F32) reinterpret_cast<float4 *>(model32)[i] = pp[u];
            if constexpr (WM == SWH_BF16) {
                const uint32_t lo = (uint32_t)f32_to_bf16_bits(pp[u].x) | ((uint32_t)f32_to_bf16_bits(pp[u].y) << 16);
                const uint32_t hi = (uint32_t)f32_to_bf16_bits(pp[u].z) | ((uint32_t)f32_to_bf16_bits(pp[u].w) << 16);
                reinterpret_cast<uint2 *>(model)[i] = uint2{lo, hi};
            }
        }
    }
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * kThreads + threadIdx.x; i < N; i += stride) {
        float pp = p[i], mm = m[i], vv = v[i];
        upd(pp, mm, vv, Elem<GDT>::load(g + i), decay_at(i));
        p[i] = pp;
        m[i] = mm;
        v[i] = vv;
        if constexpr (WM == SWH_BF16) model[i] = f32_to_bf16_bits(pp);
        if constexpr (WM == SWH_F32) model32[i] = pp;
    }
}

template <int DT>
__global__ __launch_bounds__(kThreads) void accumulate_kernel(float *__restrict__ dst,
                                                              const typename Elem<DT>::T *__restrict__ src, int64_t N,
                                                              float scale) {
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < N; i += stride)
        dst[i] = fmaf(Elem<DT>::load(src + i), scale, dst[i]);
}

// TR-DPO reference sync: target = (target * keep) + alpha * src with the
// rounding points of torch's `mul_(1 - alpha)` then `add_(src, alpha=alpha)` on
// tensors of the parameter dtype (each op rounds once to that dtype); keep is
// the host's float(1 - alpha), as torch casts the Python scalar.
template <int DT>
__global__ __launch_bounds__(kThreads) void ema_mix_kernel(typename Elem<DT>::T *__restrict__ dst,
                                                           const typename Elem<DT>::T *__restrict__ src, int64_t N,
                                                           float keep, float alpha) {
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < N; i += stride) {
        const float t = Elem<DT>::round(Elem<DT>::load(dst + i) * keep);
        const float r = fmaf(alpha, Elem<DT>::load(src + i), t);
        if constexpr (DT == SWH_F32) dst[i] = r;
        else dst[i] = f32_to_bf16_bits(r);
    }
}

// Split-K weight-gradient fold: grad = round(grad + sum_s parts[s]) with the S
// partial products (parts dtype = grad dtype) summed in fp32 in s order — the
// batched-GEMM partials of a token-split dW GEMM reduced and accumulated in ONE
// pass (replaces a torch sum over S plus an add: two extra fp32 round trips).
template <int DT>
__global__ __launch_bounds__(kThreads) void dw_reduce_kernel(const typename Elem<DT>::T *__restrict__ parts, int S,
                                                             int64_t n, typename Elem<DT>::T *__restrict__ g) {
    using T = typename Elem<DT>::T;
    constexpr int PV = kPerVec<DT>;
    const int64_t nv = n / PV;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t v = (int64_t)blockIdx.x * kThreads + threadIdx.x; v < nv; v += stride) {
        float acc[PV], x[PV];
        unpack16<DT>(reinterpret_cast<const uint4 *>(g)[v], acc);
        float s[PV];
        unpack16<DT>(reinterpret_cast<const uint4 *>(parts)[v], s);
        for (int q = 1; q < S; ++q) {
            unpack16<DT>(reinterpret_cast<const uint4 *>(parts + (int64_t)q * n)[v], x);
#pragma unroll
            for (int k = 0; k < PV; ++k) s[k] += x[k];
        }
        if constexpr (DT == SWH_F32) {
            reinterpret_cast<float4 *>(g)[v] = float4{acc[0] + s[0], acc[1] + s[1], acc[2] + s[2], acc[3] + s[3]};
        } else {
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                o[k] = (uint32_t)f32_to_bf16_bits(acc[2 * k] + s[2 * k]) |
                       ((uint32_t)f32_to_bf16_bits(acc[2 * k + 1] + s[2 * k + 1]) << 16);
            reinterpret_cast<uint4 *>(g)[v] = uint4{o[0], o[1], o[2], o[3]};
        }
    }
    (void)sizeof(T);
}

unsigned grid_for(int64_t work_items) {
    int64_t g = (work_items + kThreads - 1) / kThreads;
    if (g > 256 * 16) g = 256 * 16;
    if (g < 1) g = 1;
    return (unsigned)g;
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int64_t swh_sqnorm_partials(int64_t N) {
    int64_t n = (N + kThreads * 8 - 1) / (kThreads * 8);
    if (n > kMaxPartials) n = kMaxPartials;
    return n < 1 ? 1 : n;
}

extern "C" int swh_grad_sqnorm(const void *grad, int dtype, int64_t N, float *partials, void *stream) {
    if (!grad || !partials || N < 0) return SWH_E_ARG;
    const unsigned nb = (unsigned)swh_sqnorm_partials(N);
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
    case SWH_BF16: sqnorm_kernel<SWH_BF16><<<nb, kThreads, 0, s>>>(static_cast<const uint16_t *>(grad), N, partials); break;
    case SWH_F16: sqnorm_kernel<SWH_F16><<<nb, kThreads, 0, s>>>(static_cast<const uint16_t *>(grad), N, partials); break;
    case SWH_F32: sqnorm_kernel<SWH_F32><<<nb, kThreads, 0, s>>>(static_cast<const float *>(grad), N, partials); break;
    default: return SWH_E_DTYPE;
    }
    return launch_status();
}

extern "C" int swh_finalize_clip(const float *partials, int64_t n_partials, float max_norm, float *out2,
                                 void *stream) {
    if (!partials || !out2 || n_partials <= 0) return SWH_E_ARG;
    finalize_clip_kernel<<<1, kThreads, 0, static_cast<hipStream_t>(stream)>>>(partials, n_partials, max_norm, out2);
    return launch_status();
}

extern "C" int swh_adamw(float *master, float *exp_avg, float *exp_avg_sq, const void *grad, int grad_dtype,
                         void *model_out, int model_dtype, int64_t N, float lr, float beta1, float beta2, float eps,
                         float weight_decay, int64_t step_count, const float *clip, const int64_t *no_decay,
                         int32_t n_no_decay, void *stream) {
    if (!master || !exp_avg || !exp_avg_sq || !grad || N < 0 || step_count < 1) return SWH_E_ARG;
    if (((uintptr_t)master | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15) return SWH_E_ARG;
    if (n_no_decay < 0 || n_no_decay > kMaxNoDecay || (n_no_decay > 0 && !no_decay)) return SWH_E_ARG;
    if (model_out && model_dtype != SWH_BF16 && model_dtype != SWH_F32) return SWH_E_DTYPE;
    if (grad_dtype != SWH_BF16 && grad_dtype != SWH_F32) return SWH_E_DTYPE;
    if (N == 0) return SWH_OK;
    if ((uintptr_t)grad & (grad_dtype == SWH_BF16 ? 7 : 15)) return SWH_E_ARG;
    if (model_out && ((uintptr_t)model_out & (model_dtype == SWH_BF16 ? 7 : 15))) return SWH_E_ARG;
    const double bc1 = 1.0 - pow((double)beta1, (double)step_count);
    const double bc2 = 1.0 - pow((double)beta2, (double)step_count);
    const float step_size = (float)(lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // one float4 group per thread, no grid-stride loop: at the 0.5B size (494M elements)
    // 2.51-2.57 ms (5.4-5.5 TB/s) against 2.92-3.01 ms with 4096 looping workgroups
    // (tools/bench_adamw.py, profiles/r6_adamw_grid.log); the update is elementwise, so
    // the result does not depend on the grid
    const int64_t nbl = ((N + 3) / 4 + kThreads - 1) / kThreads;
    const unsigned nb = (unsigned)(nbl < (int64_t)INT32_MAX ? nbl : (int64_t)INT32_MAX);
    const bool nr = n_no_decay > 0 && weight_decay != 0.f;
    const int wm = model_out ? model_dtype : -1;
#define SWH_ADAM(GDT, WM, NR)                                                                                       \
    adamw_kernel<GDT, WM, NR><<<nb, kThreads, 0, s>>>(master, exp_avg, exp_avg_sq,                                 \
                                                      static_cast<const typename Elem<GDT>::T *>(grad),              \
                                                      static_cast<uint16_t *>(model_out), static_cast<float *>(model_out), N, \
                                                      lr, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt, clip, \
                                                      no_decay, n_no_decay)
#define SWH_ADAM_G(GDT)                                     \
    if (wm == SWH_BF16) {                                   \
        if (nr) SWH_ADAM(GDT, SWH_BF16, true); else SWH_ADAM(GDT, SWH_BF16, false); \
    } else if (wm == SWH_F32) {                             \
        if (nr) SWH_ADAM(GDT, SWH_F32, true); else SWH_ADAM(GDT, SWH_F32, false);   \
    } else {                                                \
        if (nr) SWH_ADAM(GDT, -1, true); else SWH_ADAM(GDT, -1, false);             \
    }
    if (grad_dtype == SWH_BF16) {
        SWH_ADAM_G(SWH_BF16)
    } else {
        SWH_ADAM_G(SWH_F32)
    }
#undef SWH_ADAM_G
#undef SWH_ADAM
    return launch_status();
}

extern "C" int swh_accumulate(float *dst, const void *src, int dtype, int64_t N, float scale, void *stream) {
    if (!dst || !src || N < 0) return SWH_E_ARG;
    if (N == 0) return SWH_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const unsigned nb = grid_for(N);
    switch (dtype) {
    case SWH_BF16: accumulate_kernel<SWH_BF16><<<nb, kThreads, 0, s>>>(dst, static_cast<const uint16_t *>(src), N, scale); break;
    case SWH_F32: accumulate_kernel<SWH_F32><<<nb, kThreads, 0, s>>>(dst, static_cast<const float *>(src), N, scale); break;
    default: return SWH_E_DTYPE;
    }
    return launch_status();
}

extern "C" int swh_ema_mix(void *target, const void *src, int dtype, int64_t N, float keep, float alpha,
                           void *stream) {
    if (!target || !src || N < 0) return SWH_E_ARG;
    if (N == 0) return SWH_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const unsigned nb = grid_for(N);
    switch (dtype) {
    case SWH_BF16: ema_mix_kernel<SWH_BF16><<<nb, kThreads, 0, s>>>(static_cast<uint16_t *>(target), static_cast<const uint16_t *>(src), N, keep, alpha); break;
    case SWH_F32: ema_mix_kernel<SWH_F32><<<nb, kThreads, 0, s>>>(static_cast<float *>(target), static_cast<const float *>(src), N, keep, alpha); break;
    default: return SWH_E_DTYPE;
    }
    return launch_status();
}

extern "C" int swh_dw_reduce(const void *parts, int32_t S, int64_t n, void *grad, int32_t dtype, void *stream) {
    if (!parts || !grad || S < 1 || n < 0) return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F32) return SWH_E_DTYPE;
    const int pv = dtype == SWH_F32 ? 4 : 8;
    if (n % pv || ((reinterpret_cast<uintptr_t>(parts) | reinterpret_cast<uintptr_t>(grad)) & 15)) return SWH_E_ARG;
    if (n == 0) return SWH_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const unsigned nb = grid_for(n / pv);
    if (dtype == SWH_BF16)
        dw_reduce_kernel<SWH_BF16><<<nb, kThreads, 0, s>>>(static_cast<const uint16_t *>(parts), S, n,
                                                           static_cast<uint16_t *>(grad));
    else
        dw_reduce_kernel<SWH_F32><<<nb, kThreads, 0, s>>>(static_cast<const float *>(parts), S, n,
                                                          static_cast<float *>(grad));
    return launch_status();
}
