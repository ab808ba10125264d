// Decoder kernels of the rollout engine (everything between the GEMMs).
//
// The reference runs transformers' Qwen2 / Llama modeling code (third-party,
// reached through grpo_trainer.py:1804 `unwrapped_model.generate` and the
// scoring forward :1249).  GEMMs stay on hipBLASLt (MFMA); these kernels
// replace the elementwise / normalisation / attention-decode ops and
// reproduce the bf16 rounding points of the transformers modules:
//   RMSNorm: bf16(w * bf16(x * rsqrt(mean(x^2) + eps)))   (Qwen2RMSNorm)
//   residual add in bf16; SiLU-gate: bf16(bf16(silu(g)) * u)
//   RoPE: bf16(bf16(q*cos) + bf16(rotate_half(q)*sin)) with bf16 cos/sin
#include "common.hpp"

namespace swh {
namespace {

// ---------------------------------------------------------------------------
// RMSNorm (+ fused residual add).  One wave per row, 4 rows per block.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const uint16_t *__restrict__ x,
                                                          const uint16_t *__restrict__ res,
                                                          uint16_t *__restrict__ res_out,
                                                          const uint16_t *__restrict__ w, int64_t rows, int64_t H,
                                                          float eps, uint16_t *__restrict__ y,
                                                          float *__restrict__ rstd_out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const uint16_t *xr = x + r * H;
    const uint16_t *rr = res ? res + r * H : nullptr;
    float ss = 0.f;
    const int64_t nv = H / 8;  // host guarantees H % 8 == 0
    for (int64_t v = lane; v < nv; v += 64) {
        float a[8];
        unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(xr)[v], a);
        if (rr) {
            float b[8];
            unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(rr)[v], b);
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = round_bf16(a[k] + b[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                o[k] = (uint32_t)f32_to_bf16_bits(a[2 * k]) | ((uint32_t)f32_to_bf16_bits(a[2 * k + 1]) << 16);
            if (res_out) reinterpret_cast<uint4 *>(res_out + r * H)[v] = uint4{o[0], o[1], o[2], o[3]};
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) ss = fmaf(a[k], a[k], ss);
    }
    ss = wave_sum(ss);
    const float rs = rsqrtf(ss / (float)H + eps);
    if (lane == 0 && rstd_out) rstd_out[r] = rs;
    const uint16_t *src = (rr && res_out) ? res_out + r * H : xr;
    for (int64_t v = lane; v < nv; v += 64) {
        float a[8], ww[8];
        if (rr && !res_out) {
            float b[8];
            unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(xr)[v], a);
            unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(rr)[v], b);
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = round_bf16(a[k] + b[k]);
        } else {
            unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(src)[v], a);
        }
        unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(w)[v], ww);
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float y0 = ww[2 * k] * round_bf16(a[2 * k] * rs);
            const float y1 = ww[2 * k + 1] * round_bf16(a[2 * k + 1] * rs);
            o[k] = (uint32_t)f32_to_bf16_bits(y0) | ((uint32_t)f32_to_bf16_bits(y1) << 16);
        }
        reinterpret_cast<uint4 *>(y + r * H)[v] = uint4{o[0], o[1], o[2], o[3]};
    }
}

// Backward.  Pass 1 (wave per row): c_r = mean(dy*w*n).  Pass 2 (thread per
// column, loop over the block's rows): dx and the dw partial of this block.
constexpr int kNormBwdThreads = 256;
__global__ __launch_bounds__(kNormBwdThreads) void rmsnorm_bwd_kernel(
    const uint16_t *__restrict__ x, const uint16_t *__restrict__ w, const float *__restrict__ rstd,
    const uint16_t *__restrict__ dy, int64_t rows, int64_t H, uint16_t *__restrict__ dx,
    float *__restrict__ dw_part, int64_t rpb) {
    extern __shared__ float cvals[];  // [rpb]
    const int64_t r0 = (int64_t)blockIdx.x * rpb;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int64_t i = wid; i < rpb; i += kNormBwdThreads / 64) {
        const int64_t r = r0 + i;
        float c = 0.f;
        if (r < rows) {
            const float rs = rstd[r];
            for (int64_t h = lane; h < H; h += 64) {
                const float n = bf16_bits_to_f32(x[r * H + h]) * rs;
                c = fmaf(bf16_bits_to_f32(dy[r * H + h]) * bf16_bits_to_f32(w[h]), n, c);
            }
        }
        c = wave_sum(c);
        if (lane == 0) cvals[i] = c / (float)H;
    }
    __syncthreads();
    for (int64_t h = threadIdx.x; h < H; h += kNormBwdThreads) {
        const float wh = bf16_bits_to_f32(w[h]);
        float dwa = 0.f;
        for (int64_t i = 0; i < rpb; ++i) {
            const int64_t r = r0 + i;
            if (r >= rows) break;
            const float rs = rstd[r];
            const float xv = bf16_bits_to_f32(x[r * H + h]);
            const float n = xv * rs;
            const float g = bf16_bits_to_f32(dy[r * H + h]);
            dx[r * H + h] = f32_to_bf16_bits(rs * (g * wh - n * cvals[i]));
            dwa = fmaf(g, round_bf16(n), dwa);
        }
        dw_part[(int64_t)blockIdx.x * H + h] = dwa;
    }
}

// ---------------------------------------------------------------------------
// SiLU gate: out = bf16(bf16(silu(g)) * u), g = gu[:, :I], u = gu[:, I:]
// ---------------------------------------------------------------------------
__device__ __forceinline__ float silu_f(float g) { return g / (1.f + expf(-g)); }

__global__ __launch_bounds__(256) void silu_mul_fwd_kernel(const uint16_t *__restrict__ gu, int64_t rows, int64_t I,
                                                           uint16_t *__restrict__ out) {
    const int64_t nv = I / 8;
    const int64_t total = rows * nv;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = idx / nv, v = idx - r * nv;
        float g[8], u[8];
        unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(gu + r * 2 * I)[v], g);
        unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(gu + r * 2 * I + I)[v], u);
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float a0 = round_bf16(silu_f(g[2 * k])) * u[2 * k];
            const float a1 = round_bf16(silu_f(g[2 * k + 1])) * u[2 * k + 1];
            o[k] = (uint32_t)f32_to_bf16_bits(a0) | ((uint32_t)f32_to_bf16_bits(a1) << 16);
        }
        reinterpret_cast<uint4 *>(out + r * I)[v] = uint4{o[0], o[1], o[2], o[3]};
    }
}

__global__ __launch_bounds__(256) void silu_mul_bwd_kernel(const uint16_t *__restrict__ gu,
                                                           const uint16_t *__restrict__ dout, int64_t rows, int64_t I,
                                                           uint16_t *__restrict__ dgu) {
    const int64_t nv = I / 8;
    const int64_t total = rows * nv;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = idx / nv, v = idx - r * nv;
        float g[8], u[8], d[8];
        unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(gu + r * 2 * I)[v], g);
        unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(gu + r * 2 * I + I)[v], u);
        unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(dout + r * I)[v], d);
        uint32_t og[4], ou[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float rg[2], ru[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const float gg = g[2 * k + e];
                const float sg = 1.f / (1.f + expf(-gg));
                const float a = round_bf16(gg * sg);
                ru[e] = d[2 * k + e] * a;                       // d u   = dout * silu(g)
                const float ga = round_bf16(d[2 * k + e] * u[2 * k + e]);  // d silu = dout * u
                rg[e] = ga * sg * (1.f + gg * (1.f - sg));
            }
            og[k] = (uint32_t)f32_to_bf16_bits(rg[0]) | ((uint32_t)f32_to_bf16_bits(rg[1]) << 16);
            ou[k] = (uint32_t)f32_to_bf16_bits(ru[0]) | ((uint32_t)f32_to_bf16_bits(ru[1]) << 16);
        }
        reinterpret_cast<uint4 *>(dgu + r * 2 * I)[v] = uint4{og[0], og[1], og[2], og[3]};
        reinterpret_cast<uint4 *>(dgu + r * 2 * I + I)[v] = uint4{ou[0], ou[1], ou[2], ou[3]};
    }
}

__global__ __launch_bounds__(256) void embed_gather_kernel(const uint16_t *__restrict__ table,
                                                           const int64_t *__restrict__ ids, int64_t H,
                                                           uint16_t *__restrict__ x) {
    const int64_t b = blockIdx.x;
    const int64_t id = ids[b];
    const int64_t nv = H / 8;
    for (int64_t v = threadIdx.x; v < nv; v += blockDim.x)
        reinterpret_cast<uint4 *>(x + b * H)[v] = reinterpret_cast<const uint4 *>(table + id * H)[v];
}

// ---------------------------------------------------------------------------
// Attention decode (GQA), one workgroup per (kv head, sequence).
// ---------------------------------------------------------------------------
constexpr int kAttnThreads = 256;
constexpr int kTile = 256;
constexpr int kMaxGq = 16;

template <int D>
__global__ __launch_bounds__(kAttnThreads) void attn_decode_kernel(
    const uint16_t *__restrict__ qkv, uint16_t *__restrict__ kc, uint16_t *__restrict__ vc,
    const float *__restrict__ rcos, const float *__restrict__ rsin, const int32_t *__restrict__ plen,
    const int32_t *__restrict__ state, int Hq, int Hkv, int Tmax, float scale, uint16_t *__restrict__ out) {
    constexpr int LPK = D / 8;         // lanes per key (8 dims per lane)
    constexpr int KPW = 64 / LPK;      // keys per wave per iteration
    constexpr int NW = kAttnThreads / 64;
    __shared__ float q_s[kMaxGq * D];
    __shared__ float sc[kMaxGq * (kTile + 1)];
    __shared__ float m_s[kMaxGq], l_s[kMaxGq], f_s[kMaxGq];
    __shared__ uint16_t knew[D], vnew[D];

    const int kvh = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int Gq = Hq / Hkv;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // state[0] = index of the token the sampler produces in this decode step;
    // the attention input is the previous token, index state[0] - 1.
    const int step = state[0] - 1, P = state[1];
    const int pl = plen[b];
    const int slot_new = P + step;
    const int start = P - pl;
    const int pos = pl + step;
    if (step < 0 || slot_new >= Tmax || pl < 0 || pl > P) {  // never write outside the cache
        const int Gq0 = Hq / Hkv;
        for (int idx = threadIdx.x; idx < Gq0 * D; idx += kAttnThreads)
            out[b * (int64_t)Hq * D + kvh * Gq0 * D + idx] = 0x7fc0;  // NaN: fail loudly
        return;
    }
    const int W = (Hq + 2 * Hkv) * D;
    const uint16_t *row = qkv + b * (int64_t)W;
    const int64_t cbase = ((b * Hkv + kvh) * (int64_t)Tmax) * D;

    // RoPE on q (Gq heads) and the new k; v copied.  Thread i < D/2 handles pair (i, i + D/2).
    constexpr int HD = D / 2;
    for (int idx = tid; idx < (Gq + 1) * HD; idx += kAttnThreads) {
        const int hh = idx / HD, i = idx - hh * HD;
        const float c = rcos[(int64_t)pos * HD + i], s = rsin[(int64_t)pos * HD + i];
        const uint16_t *src = (hh < Gq) ? row + (kvh * Gq + hh) * D : row + (Hq + kvh) * D;
        const float x1 = bf16_bits_to_f32(src[i]), x2 = bf16_bits_to_f32(src[i + HD]);
        const float o1 = round_bf16(round_bf16(x1 * c) + round_bf16(-x2 * s));
        const float o2 = round_bf16(round_bf16(x2 * c) + round_bf16(x1 * s));
        if (hh < Gq) {
            q_s[hh * D + i] = o1;
            q_s[hh * D + i + HD] = o2;
        } else {
            knew[i] = f32_to_bf16_bits(o1);
            knew[i + HD] = f32_to_bf16_bits(o2);
        }
    }
    for (int d = tid; d < D; d += kAttnThreads) vnew[d] = row[(Hq + Hkv + kvh) * D + d];
    if (tid < kMaxGq) {
        m_s[tid] = kNegInf;
        l_s[tid] = 0.f;
    }
    __syncthreads();
    for (int d = tid; d < D; d += kAttnThreads) {
        kc[cbase + (int64_t)slot_new * D + d] = knew[d];
        vc[cbase + (int64_t)slot_new * D + d] = vnew[d];
    }

    // this lane's q slice for every head of the group
    const int part = lane % LPK, kin = lane / LPK;
    float qreg[kMaxGq][8];
#pragma unroll
    for (int h = 0; h < kMaxGq; ++h)
#pragma unroll
        for (int k = 0; k < 8; ++k) qreg[h][k] = (h < Gq) ? q_s[h * D + part * 8 + k] : 0.f;

    // output accumulators: thread owns (h, d) for idx = tid + j*256 < Gq*D
    constexpr int kAcc = (kMaxGq * D + kAttnThreads - 1) / kAttnThreads;
    float acc[kAcc];
#pragma unroll
    for (int j = 0; j < kAcc; ++j) acc[j] = 0.f;

    for (int ts = start; ts <= slot_new; ts += kTile) {
        const int te = (ts + kTile - 1 < slot_new) ? ts + kTile - 1 : slot_new;  // inclusive
        const int n = te - ts + 1;
        // phase A: scores
        for (int base = wid * KPW; base < n; base += NW * KPW) {
            const int kk = base + kin;
            float part_dot[kMaxGq];
#pragma unroll
            for (int h = 0; h < kMaxGq; ++h) part_dot[h] = 0.f;
            if (kk < n) {
                const int slot = ts + kk;
                float kv[8];
                if (slot == slot_new) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) kv[k] = bf16_bits_to_f32(knew[part * 8 + k]);
                } else {
                    unpack16<SWH_BF16>(*reinterpret_cast<const uint4 *>(kc + cbase + (int64_t)slot * D + part * 8), kv);
                }
#pragma unroll
                for (int h = 0; h < kMaxGq; ++h) {
                    float s = 0.f;
#pragma unroll
                    for (int k = 0; k < 8; ++k) s = fmaf(qreg[h][k], kv[k], s);
                    part_dot[h] = s;
                }
            }
#pragma unroll
            for (int h = 0; h < kMaxGq; ++h) {
                float s = part_dot[h];
#pragma unroll
                for (int o = 1; o < LPK; o <<= 1) s += __shfl_xor(s, o, kWave);
                part_dot[h] = s;
            }
            if (part == 0 && kk < n) {
#pragma unroll
                for (int h = 0; h < kMaxGq; ++h)
                    if (h < Gq) sc[h * (kTile + 1) + kk] = part_dot[h] * scale;
            }
        }
        __syncthreads();
        // phase B: online softmax per head
        for (int h = wid; h < Gq; h += NW) {
            float mx = kNegInf;
            for (int k = lane; k < n; k += 64) mx = fmaxf(mx, sc[h * (kTile + 1) + k]);
            mx = wave_max(mx);
            const float mo = m_s[h];
            const float mn = fmaxf(mo, mx);
            const float f = (mo == kNegInf) ? 0.f : expf(mo - mn);
            float sum = 0.f;
            for (int k = lane; k < n; k += 64) {
                const float pv = expf(sc[h * (kTile + 1) + k] - mn);
                sc[h * (kTile + 1) + k] = pv;
                sum += pv;
            }
            sum = wave_sum(sum);
            if (lane == 0) {
                m_s[h] = mn;
                l_s[h] = l_s[h] * f + sum;
                f_s[h] = f;
            }
        }
        __syncthreads();
        // phase C: P V
#pragma unroll
        for (int j = 0; j < kAcc; ++j) {
            const int idx = tid + j * kAttnThreads;
            if (idx < Gq * D) {
                const int h = idx / D, d = idx - h * D;
                float a = acc[j] * f_s[h];
                const float *ph = sc + h * (kTile + 1);
                const uint16_t *vp = vc + cbase + (int64_t)ts * D + d;
                const int nc = (te == slot_new) ? n - 1 : n;
                for (int k = 0; k < nc; ++k) a = fmaf(ph[k], bf16_bits_to_f32(vp[(int64_t)k * D]), a);
                if (nc < n) a = fmaf(ph[n - 1], bf16_bits_to_f32(vnew[d]), a);
                acc[j] = a;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < kAcc; ++j) {
        const int idx = tid + j * kAttnThreads;
        if (idx < Gq * D) {
            const int h = idx / D, d = idx - h * D;
            out[b * (int64_t)Hq * D + (kvh * Gq + h) * D + d] = f32_to_bf16_bits(acc[j] / l_s[h]);
        }
    }
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int swh_rmsnorm_fwd(const void *x, const void *residual, void *residual_out, const void *weight,
                               int64_t rows, int64_t H, float eps, void *y, float *rstd, void *stream) {
    if (!x || !weight || !y || rows < 0 || H <= 0 || H % 8) return SWH_E_ARG;
    if (rows == 0) return SWH_OK;
    rmsnorm_fwd_kernel<<<dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(x), static_cast<const uint16_t *>(residual), static_cast<uint16_t *>(residual_out),
        static_cast<const uint16_t *>(weight), rows, H, eps, static_cast<uint16_t *>(y), rstd);
    return launch_status();
}

extern "C" int swh_rmsnorm_bwd(const void *x, const void *weight, const float *rstd, const void *dy, int64_t rows,
                               int64_t H, void *dx, float *dw_partial, int64_t rows_per_block, void *stream) {
    if (!x || !weight || !rstd || !dy || !dx || !dw_partial || rows < 0 || H <= 0 || rows_per_block <= 0 ||
        rows_per_block > 4096)
        return SWH_E_ARG;
    if (rows == 0) return SWH_OK;
    const unsigned nb = (unsigned)((rows + rows_per_block - 1) / rows_per_block);
    rmsnorm_bwd_kernel<<<dim3(nb), dim3(kNormBwdThreads), rows_per_block * sizeof(float),
                         static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(x), static_cast<const uint16_t *>(weight), rstd, static_cast<const uint16_t *>(dy),
        rows, H, static_cast<uint16_t *>(dx), dw_partial, rows_per_block);
    return launch_status();
}

static unsigned ew_grid(int64_t work) {
    int64_t g = (work + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;
    return (unsigned)(g < 1 ? 1 : g);
}

extern "C" int swh_silu_mul_fwd(const void *gu, int64_t rows, int64_t I, void *out, void *stream) {
    if (!gu || !out || rows < 0 || I <= 0 || I % 8) return SWH_E_ARG;
    if (rows == 0) return SWH_OK;
    silu_mul_fwd_kernel<<<ew_grid(rows * I / 8), 256, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(gu), rows, I, static_cast<uint16_t *>(out));
    return launch_status();
}

extern "C" int swh_silu_mul_bwd(const void *gu, const void *dout, int64_t rows, int64_t I, void *dgu, void *stream) {
    if (!gu || !dout || !dgu || rows < 0 || I <= 0 || I % 8) return SWH_E_ARG;
    if (rows == 0) return SWH_OK;
    silu_mul_bwd_kernel<<<ew_grid(rows * I / 8), 256, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(gu), static_cast<const uint16_t *>(dout), rows, I, static_cast<uint16_t *>(dgu));
    return launch_status();
}

extern "C" int swh_embed_gather(const void *table, const int64_t *ids, int64_t B, int64_t H, void *x, void *stream) {
    if (!table || !ids || !x || B < 0 || H <= 0 || H % 8) return SWH_E_ARG;
    if (B == 0) return SWH_OK;
    embed_gather_kernel<<<dim3((unsigned)B), 128, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(table), ids, H, static_cast<uint16_t *>(x));
    return launch_status();
}

extern "C" int swh_attn_decode(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                               const float *rope_sin, const int32_t *prompt_len, const int32_t *state, int64_t B,
                               int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax, float scale, void *out,
                               void *stream) {
    if (!qkv || !k_cache || !v_cache || !rope_cos || !rope_sin || !prompt_len || !state || !out || B < 0 || Hkv <= 0 ||
        Hq % Hkv || Hq / Hkv > kMaxGq || Tmax <= 0)
        return SWH_E_ARG;
    if (B == 0) return SWH_OK;
    dim3 grid((unsigned)Hkv, (unsigned)B), block(kAttnThreads);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint16_t *q = static_cast<const uint16_t *>(qkv);
    uint16_t *kc = static_cast<uint16_t *>(k_cache), *vc = static_cast<uint16_t *>(v_cache);
    uint16_t *o = static_cast<uint16_t *>(out);
    if (D == 64)
        attn_decode_kernel<64><<<grid, block, 0, s>>>(q, kc, vc, rope_cos, rope_sin, prompt_len, state, Hq, Hkv, Tmax,
                                                      scale, o);
    else if (D == 128)
        attn_decode_kernel<128><<<grid, block, 0, s>>>(q, kc, vc, rope_cos, rope_sin, prompt_len, state, Hq, Hkv, Tmax,
                                                       scale, o);
    else
        return SWH_E_ARG;
    return launch_status();
}
