// GPT-2 family kernels (BASELINE.json config 1: tiny GPT-2 plumbing): the
// LayerNorm (with bias, optionally fused with the residual add that precedes
// it) and the tanh-approximated GELU ("gelu_new") of transformers' GPT2Model,
// forward and backward, bf16 or fp32.  The projections are library GEMMs and
// the attention torch SDPA (head_dim 16 at config 1 is below the MFMA
// attention tile), as in the fp32 reference-precision mode of the Qwen2 /
// Llama path.
//
// Rounding points follow the torch ops transformers runs:
//   residual: s = dtype(x + r)                    (GPT2Block `residual + h`)
//   LayerNorm: fp32 mean / biased variance / rstd, y = dtype((s - mean) rstd w + b)
//   gelu_new: 0.5 * x * (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))), one dtype
//             rounding per torch op of NewGELUActivation (pow = two
//             multiplies, mul, add, mul, tanh, add, mul, mul) — none for fp32.
// HBM-bound elementwise / row work: a few passes over rows x H.
#include "common.hpp"

namespace swh {
namespace {

template <int DT> __device__ __forceinline__ void store_elem(typename Elem<DT>::T *p, float v) {
    if constexpr (DT == SWH_F32) *p = v;
    else *p = f32_to_bf16_bits(v);
}

// One wave per row, four rows per workgroup.
template <int DT>
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const typename Elem<DT>::T *__restrict__ x,
                                                            const typename Elem<DT>::T *__restrict__ r,
                                                            const typename Elem<DT>::T *__restrict__ w,
                                                            const typename Elem<DT>::T *__restrict__ b, int64_t rows,
                                                            int64_t H, float eps, typename Elem<DT>::T *__restrict__ y,
                                                            typename Elem<DT>::T *__restrict__ s_out,
                                                            float *__restrict__ mean_out, float *__restrict__ rstd_out) {
    using T = typename Elem<DT>::T;
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const T *xr = x + row * H;
    const T *rr = r ? r + row * H : nullptr;
    T *sr = s_out ? s_out + row * H : nullptr;
    auto val = [&](int64_t c) -> float {
        const float v = Elem<DT>::load(xr + c);
        return rr ? Elem<DT>::round(v + Elem<DT>::load(rr + c)) : v;
    };
    float sum = 0.f;
    for (int64_t c = lane; c < H; c += 64) {
        const float v = val(c);
        if (sr) store_elem<DT>(sr + c, v);
        sum += v;
    }
    const float mean = wave_sum(sum) / (float)H;
    float sq = 0.f;
    for (int64_t c = lane; c < H; c += 64) {
        const float d = val(c) - mean;
        sq = fmaf(d, d, sq);
    }
    const float rstd = rsqrtf(wave_sum(sq) / (float)H + eps);
    T *yr = y + row * H;
    for (int64_t c = lane; c < H; c += 64) {
        const float v = (val(c) - mean) * rstd;
        store_elem<DT>(yr + c, fmaf(v, Elem<DT>::load(w + c), Elem<DT>::load(b + c)));
    }
    if (lane == 0) {
        mean_out[row] = mean;
        rstd_out[row] = rstd;
    }
}

// dx = rstd (g - mean(g) - xhat mean(g xhat)) (+ dres), g = dy w, one wave per row.
template <int DT>
__global__ __launch_bounds__(256) void layernorm_bwd_dx_kernel(const typename Elem<DT>::T *__restrict__ s,
                                                               const typename Elem<DT>::T *__restrict__ w,
                                                               const float *__restrict__ mean,
                                                               const float *__restrict__ rstd,
                                                               const typename Elem<DT>::T *__restrict__ dy,
                                                               const typename Elem<DT>::T *__restrict__ dres,
                                                               int64_t rows, int64_t H,
                                                               typename Elem<DT>::T *__restrict__ dx) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float mu = mean[row], rs = rstd[row];
    const int64_t o = row * H;
    float a = 0.f, bb = 0.f;
    for (int64_t c = lane; c < H; c += 64) {
        const float g = Elem<DT>::load(dy + o + c) * Elem<DT>::load(w + c);
        const float xh = (Elem<DT>::load(s + o + c) - mu) * rs;
        a += g;
        bb = fmaf(g, xh, bb);
    }
    a = wave_sum(a) / (float)H;
    bb = wave_sum(bb) / (float)H;
    for (int64_t c = lane; c < H; c += 64) {
        const float g = Elem<DT>::load(dy + o + c) * Elem<DT>::load(w + c);
        const float xh = (Elem<DT>::load(s + o + c) - mu) * rs;
        float v = rs * (g - a - xh * bb);
        if (dres) v += Elem<DT>::load(dres + o + c);
        store_elem<DT>(dx + o + c, v);
    }
}

// Weight / bias gradient partials: one thread per column over a block of rows,
// in fixed row order: part_w[blk][c] = sum dy xhat, part_b[blk][c] = sum dy.
template <int DT>
__global__ __launch_bounds__(256) void layernorm_bwd_dwb_kernel(const typename Elem<DT>::T *__restrict__ s,
                                                                const float *__restrict__ mean,
                                                                const float *__restrict__ rstd,
                                                                const typename Elem<DT>::T *__restrict__ dy,
                                                                int64_t rows, int64_t H, int64_t rpb,
                                                                float *__restrict__ part_w, float *__restrict__ part_b) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= H) return;
    const int64_t r0 = (int64_t)blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
    float pw = 0.f, pb = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        const float g = Elem<DT>::load(dy + r * H + c);
        pw = fmaf(g, (Elem<DT>::load(s + r * H + c) - mean[r]) * rstd[r], pw);
        pb += g;
    }
    part_w[blockIdx.y * H + c] = pw;
    part_b[blockIdx.y * H + c] = pb;
}

constexpr float kGeluK = 0.7978845608028654f;  // sqrt(2 / pi)
constexpr float kGeluC = 0.044715f;

template <int DT> __device__ __forceinline__ float gelu_new(float x) {
    auto rd = [](float v) { return Elem<DT>::round(v); };
    const float p = rd(rd(x * x) * x);            // torch.pow(x, 3.0): base * base * base in the dtype
    const float inner = rd(x + rd(kGeluC * p));   // x + 0.044715 * pow
    const float t = rd(tanhf(rd(kGeluK * inner)));
    return rd(rd(0.5f * x) * rd(1.f + t));        // (0.5 * x) * (1 + tanh(...))
}

template <int DT>
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const typename Elem<DT>::T *__restrict__ x, int64_t n,
                                                       typename Elem<DT>::T *__restrict__ y) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        store_elem<DT>(y + i, gelu_new<DT>(Elem<DT>::load(x + i)));
}

// d gelu_new / dx = 0.5 (1 + t) + 0.5 x (1 - t^2) sqrt(2/pi) (1 + 3 c x^2), fp32 math
template <int DT>
__global__ __launch_bounds__(256) void gelu_bwd_kernel(const typename Elem<DT>::T *__restrict__ x,
                                                       const typename Elem<DT>::T *__restrict__ dy, int64_t n,
                                                       typename Elem<DT>::T *__restrict__ dx) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float v = Elem<DT>::load(x + i);
        const float t = tanhf(kGeluK * (v + kGeluC * v * v * v));
        const float d = 0.5f * (1.f + t) + 0.5f * v * (1.f - t * t) * kGeluK * (1.f + 3.f * kGeluC * v * v);
        store_elem<DT>(dx + i, Elem<DT>::load(dy + i) * d);
    }
}

unsigned ew_blocks(int64_t n) {
    int64_t g = (n + 255) / 256;
    if (g > 256 * 32) g = 256 * 32;
    return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace
}  // namespace swh

using namespace swh;

// the launch statement(s) in __VA_ARGS__ see DT (dtype code) and T (element type)
#define SWH_DT_DISPATCH(dtype, ...)                                    \
    do {                                                               \
        if ((dtype) == SWH_BF16) {                                     \
            constexpr int DT = SWH_BF16;                               \
            using T = uint16_t;                                        \
            __VA_ARGS__;                                               \
        } else if ((dtype) == SWH_F32) {                               \
            constexpr int DT = SWH_F32;                                \
            using T = float;                                           \
            __VA_ARGS__;                                               \
        } else {                                                       \
            return SWH_E_DTYPE;                                        \
        }                                                              \
    } while (0)

extern "C" int swh_layernorm_fwd(const void *x, const void *residual, const void *w, const void *b, int64_t rows,
                                 int64_t H, float eps, void *y, void *s_out, float *mean, float *rstd, int32_t dtype,
                                 void *stream) {
    if (!x || !w || !b || !y || !mean || !rstd || rows < 0 || H <= 0 || (residual && !s_out)) return SWH_E_ARG;
    if (rows == 0) return SWH_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((rows + 3) / 4));
    SWH_DT_DISPATCH(dtype, layernorm_fwd_kernel<DT><<<grid, 256, 0, st>>>(
                               static_cast<const T *>(x), static_cast<const T *>(residual), static_cast<const T *>(w),
                               static_cast<const T *>(b), rows, H, eps, static_cast<T *>(y), static_cast<T *>(s_out),
                               mean, rstd));
    return launch_status();
}

extern "C" int64_t swh_layernorm_bwd_partial_rows(int64_t rows, int64_t rows_per_block) {
    return rows <= 0 || rows_per_block <= 0 ? 0 : (rows + rows_per_block - 1) / rows_per_block;
}

extern "C" int swh_layernorm_bwd(const void *s, const void *w, const float *mean, const float *rstd, const void *dy,
                                 const void *dres, int64_t rows, int64_t H, int64_t rows_per_block, void *dx,
                                 float *part_w, float *part_b, int32_t dtype, void *stream) {
    if (!s || !w || !mean || !rstd || !dy || !dx || rows < 0 || H <= 0 || rows_per_block <= 0 || (!part_w != !part_b))
        return SWH_E_ARG;
    if (rows == 0) return SWH_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((rows + 3) / 4));
    const dim3 gp((unsigned)((H + 255) / 256), (unsigned)((rows + rows_per_block - 1) / rows_per_block));
    SWH_DT_DISPATCH(dtype, layernorm_bwd_dx_kernel<DT><<<grid, 256, 0, st>>>(
                               static_cast<const T *>(s), static_cast<const T *>(w), mean, rstd,
                               static_cast<const T *>(dy), static_cast<const T *>(dres), rows, H, static_cast<T *>(dx)));
    if (part_w)
        SWH_DT_DISPATCH(dtype, layernorm_bwd_dwb_kernel<DT><<<gp, 256, 0, st>>>(
                                   static_cast<const T *>(s), mean, rstd, static_cast<const T *>(dy), rows, H,
                                   rows_per_block, part_w, part_b));
    return launch_status();
}

extern "C" int swh_gelu_tanh_fwd(const void *x, int64_t n, void *y, int32_t dtype, void *stream) {
    if (!x || !y || n < 0) return SWH_E_ARG;
    if (n == 0) return SWH_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    SWH_DT_DISPATCH(dtype, gelu_fwd_kernel<DT><<<ew_blocks(n), 256, 0, st>>>(static_cast<const T *>(x), n,
                                                                              static_cast<T *>(y)));
    return launch_status();
}

extern "C" int swh_gelu_tanh_bwd(const void *x, const void *dy, int64_t n, void *dx, int32_t dtype, void *stream) {
    if (!x || !dy || !dx || n < 0) return SWH_E_ARG;
    if (n == 0) return SWH_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    SWH_DT_DISPATCH(dtype, gelu_bwd_kernel<DT><<<ew_blocks(n), 256, 0, st>>>(
                               static_cast<const T *>(x), static_cast<const T *>(dy), n, static_cast<T *>(dx)));
    return launch_status();
}
