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

// Backward, one pass: a wave owns whole rows (16-B loads, the row stays in
// registers): c_r = mean(dy*w*n), dx = rstd*(dy*w - n*c_r), and each lane
// accumulates dw = sum dy*bf16(n) for its columns over the wave's rows; the
// block's waves meet in LDS and write one dw partial row per block.
constexpr int kNormBwdThreads = 256;
constexpr int kNormBwdVec = 8;  // max 16-B vectors per lane per row: H <= 64 * 8 * 8 = 4096
template <int VEC>
__global__ __launch_bounds__(kNormBwdThreads) void rmsnorm_bwd_kernel(
    const uint16_t *__restrict__ x, const uint16_t *__restrict__ w, const float *__restrict__ rstd,
    const uint16_t *__restrict__ dy, int64_t rows, int64_t H, uint16_t *__restrict__ dx,
    float *__restrict__ dw_part, int64_t rpb, const uint16_t *__restrict__ dres) {
    extern __shared__ float dws[];  // [waves][H]
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NWV = kNormBwdThreads / 64;
    const int nv = (int)(H / 8);
    const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
    float wv[VEC][8], dwa[VEC][8];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        const int v = lane + 64 * j;
        if (v < nv) unpack16<SWH_BF16>(reinterpret_cast<const uint4 *>(w)[v], wv[j]);
#pragma unroll
        for (int k = 0; k < 8; ++k) dwa[j][k] = 0.f;
    }
    // a row's x / dy / dres (and rstd) are loaded one row ahead: the next row's loads
    // are in flight while this row reduces and stores
    uint4 nx[VEC], ng[VEC], nd[VEC];
    float nrs = 0.f;
    auto load_row = [&](int64_t r) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            const int v = lane + 64 * j;
            if (v < nv) {
                nx[j] = reinterpret_cast<const uint4 *>(x + r * H)[v];
                ng[j] = reinterpret_cast<const uint4 *>(dy + r * H)[v];
                if (dres) nd[j] = reinterpret_cast<const uint4 *>(dres + r * H)[v];
            }
        }
        nrs = rstd[r];
    };
    if (r0 + wid < r1) load_row(r0 + wid);
    for (int64_t r = r0 + wid; r < r1; r += NWV) {
        uint4 xv[VEC], gv[VEC], dv[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            xv[j] = nx[j];
            gv[j] = ng[j];
            dv[j] = nd[j];
        }
        const float rs = nrs;
        if (r + NWV < r1) load_row(r + NWV);
        float c = 0.f;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            if (lane + 64 * j < nv) {
                float a[8], g[8];
                unpack16<SWH_BF16>(xv[j], a);
                unpack16<SWH_BF16>(gv[j], g);
#pragma unroll
                for (int k = 0; k < 8; ++k) c = fmaf(g[k] * wv[j][k], a[k] * rs, c);
            }
        }
        c = wave_sum(c) / (float)H;
        uint4 *dxr = reinterpret_cast<uint4 *>(dx + r * H);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            if (lane + 64 * j < nv) {
                float a[8], g[8];
                unpack16<SWH_BF16>(xv[j], a);
                unpack16<SWH_BF16>(gv[j], g);
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float n = a[k] * rs;
                    dwa[j][k] = fmaf(g[k], round_bf16(n), dwa[j][k]);
                    a[k] = rs * (g[k] * wv[j][k] - n * c);
                }
                if (dres) {  // + the residual branch's gradient: bf16(bf16(dx_norm) + dres), as autograd adds them
                    float d[8];
                    unpack16<SWH_BF16>(dv[j], d);
#pragma unroll
                    for (int k = 0; k < 8; ++k) a[k] = round_bf16(a[k]) + d[k];
                }
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    o[k] = (uint32_t)f32_to_bf16_bits(a[2 * k]) | ((uint32_t)f32_to_bf16_bits(a[2 * k + 1]) << 16);
                dxr[lane + 64 * j] = uint4{o[0], o[1], o[2], o[3]};
            }
        }
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
        const int v = lane + 64 * j;
        if (v < nv) {
#pragma unroll
            for (int k = 0; k < 8; ++k) dws[wid * H + v * 8 + k] = dwa[j][k];
        }
    }
    __syncthreads();
    for (int64_t h = threadIdx.x; h < H; h += kNormBwdThreads) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NWV; ++q) t += dws[q * H + h];
        dw_part[(int64_t)blockIdx.x * H + h] = t;
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

// Folded RMSNorm weights for the decode GEMMs, all matrices in one launch:
// out_j[n][k] = bf16(W_j[n][k] * w_j[k]) (the product torch's bf16 mul forms).
// Job table in device memory: {W, w, out, N, K} per matrix; the grid strides
// over the concatenated rows.
struct FoldJob {
    const uint16_t *w;
    const uint16_t *nw;
    uint16_t *out;
    int64_t rows, cols;
    int64_t row0;  // first global row of this job
};

constexpr int kFoldMaxJobs = 256, kFoldRows = 8;
// a workgroup folds chunks of kFoldRows rows; the job table is read into LDS once
// and a chunk finds its job by binary search there.  A chunk inside one job is one
// flat run of 16-B pieces (every thread's loads issued together); a chunk that
// straddles jobs goes row by row.
__global__ __launch_bounds__(256) void fold_norm_kernel(const FoldJob *__restrict__ jobs, int njobs,
                                                        int64_t total_rows) {
    __shared__ FoldJob tab[kFoldMaxJobs];
    for (int j = threadIdx.x; j < njobs; j += blockDim.x) tab[j] = jobs[j];
    __syncthreads();
    auto find = [&](int64_t gr) {
        int lo = 0, hi = njobs - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (tab[mid].row0 <= gr) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    auto fold8 = [](const uint4 &x, const uint4 &w) {
        float a[8], b[8];
        unpack16<SWH_BF16>(x, a);
        unpack16<SWH_BF16>(w, b);
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            o[q] = (uint32_t)f32_to_bf16_bits(a[2 * q] * b[2 * q]) |
                   ((uint32_t)f32_to_bf16_bits(a[2 * q + 1] * b[2 * q + 1]) << 16);
        return uint4{o[0], o[1], o[2], o[3]};
    };
    const int64_t nchunk = (total_rows + kFoldRows - 1) / kFoldRows;
    for (int64_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
        const int64_t g0 = ch * kFoldRows, g1 = min(g0 + kFoldRows, total_rows);
        const int j = find(g0);
        const FoldJob &jb = tab[j];
        if (g1 <= jb.row0 + jb.rows) {  // one job: a flat run of (g1 - g0) * cols / 8 pieces
            const int64_t cpr = jb.cols / 8, np = (g1 - g0) * cpr;
            const uint4 *src = reinterpret_cast<const uint4 *>(jb.w + (g0 - jb.row0) * jb.cols);
            const uint4 *nv = reinterpret_cast<const uint4 *>(jb.nw);
            uint4 *dst = reinterpret_cast<uint4 *>(jb.out + (g0 - jb.row0) * jb.cols);
            for (int64_t p0 = threadIdx.x; p0 < np; p0 += 4 * blockDim.x) {
                uint4 x[4], w[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int64_t p = p0 + u * blockDim.x;
                    if (p < np) {
                        x[u] = src[p];
                        w[u] = nv[p % cpr];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int64_t p = p0 + u * blockDim.x;
                    if (p < np) dst[p] = fold8(x[u], w[u]);
                }
            }
        } else {
            for (int64_t gr = g0; gr < g1; ++gr) {
                const FoldJob &jr = tab[find(gr)];
                const int64_t r = gr - jr.row0;
                const uint4 *src = reinterpret_cast<const uint4 *>(jr.w + r * jr.cols);
                const uint4 *nv = reinterpret_cast<const uint4 *>(jr.nw);
                uint4 *dst = reinterpret_cast<uint4 *>(jr.out + r * jr.cols);
                for (int64_t c = threadIdx.x; c < jr.cols / 8; c += blockDim.x) dst[c] = fold8(src[c], nv[c]);
            }
        }
    }
}

// ss_out (nullable): per 16-column chunk sums of squares of the gathered row,
// the RMSNorm statistic the decode GEMM prologue consumes (swh_decode_gemm ss_in)
__global__ __launch_bounds__(256) void embed_gather_kernel(const uint16_t *__restrict__ table,
                                                           const int64_t *__restrict__ ids, int64_t H,
                                                           uint16_t *__restrict__ x, float *__restrict__ ss_out) {
    const int64_t b = blockIdx.x;
    const int64_t id = ids[b];
    const int64_t nch = H / 16;
    for (int64_t c = threadIdx.x; c < nch; c += blockDim.x) {
        const uint4 *src = reinterpret_cast<const uint4 *>(table + id * H) + 2 * c;
        const uint4 lo = src[0], hi = src[1];
        uint4 *dst = reinterpret_cast<uint4 *>(x + b * H) + 2 * c;
        dst[0] = lo;
        dst[1] = hi;
        if (ss_out) {
            float a[8], e[8];
            unpack16<SWH_BF16>(lo, a);
            unpack16<SWH_BF16>(hi, e);
            float ss = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) ss = fmaf(a[k], a[k], ss);
#pragma unroll
            for (int k = 0; k < 8; ++k) ss = fmaf(e[k], e[k], ss);
            ss_out[b * nch + c] = ss;
        }
    }
}

// ---------------------------------------------------------------------------
// QKV split + RoPE for the full-sequence forward (training / prefill):
// qkv [R = B*L, (Hq + 2 Hkv) D] -> q [B, Hq, L, D], k [B, Hkv, L, D] (rotated),
// v [B, Hkv, L, D]; transformers' bf16 rotate-half: y1 = bf16(bf16(x1 c) +
// bf16(-x2 s)), y2 = bf16(bf16(x2 c) + bf16(x1 s)).  One thread = 8 pairs.
// Backward (torch autograd of those bf16 ops): dx1 = bf16(bf16(dy1 c) +
// bf16(dy2 s)), dx2 = bf16(bf16(dy2 c) - bf16(dy1 s)); v passes through.
// ---------------------------------------------------------------------------
template <bool BWD>
__global__ __launch_bounds__(256) void qkv_rope_kernel(uint16_t *__restrict__ qkv, const int64_t *__restrict__ pos,
                                                       const float *__restrict__ rc, const float *__restrict__ rs,
                                                       int64_t R, int L, int Hq, int Hkv, int D,
                                                       uint16_t *__restrict__ q, uint16_t *__restrict__ k,
                                                       uint16_t *__restrict__ v) {
    const int HD = D / 2, G = HD / 8;  // 8-pair groups per head
    const int H3 = Hq + 2 * Hkv;
    const int64_t total = R * H3 * G;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int gi = (int)(idx % G);
        const int h = (int)((idx / G) % H3);
        const int64_t r = idx / ((int64_t)G * H3);
        const int64_t b = r / L, l = r - b * L;
        uint16_t *src = qkv + r * (int64_t)H3 * D + (int64_t)h * D + gi * 8;
        uint16_t *dst;
        if (h < Hq) dst = q + ((b * Hq + h) * (int64_t)L + l) * D + gi * 8;
        else if (h < Hq + Hkv) dst = k + ((b * Hkv + (h - Hq)) * (int64_t)L + l) * D + gi * 8;
        else dst = v + ((b * Hkv + (h - Hq - Hkv)) * (int64_t)L + l) * D + gi * 8;
        uint4 *a1 = reinterpret_cast<uint4 *>(BWD ? src : dst), *a2 = reinterpret_cast<uint4 *>((BWD ? src : dst) + HD);
        const uint4 *i1 = reinterpret_cast<const uint4 *>(BWD ? dst : src);
        const uint4 *i2 = reinterpret_cast<const uint4 *>((BWD ? dst : src) + HD);
        if (h >= Hq + Hkv) {  // v: copy
            *a1 = *i1;
            *a2 = *i2;
            continue;
        }
        const int64_t p = pos[r] < 0 ? 0 : pos[r];
        const float4 *cp = reinterpret_cast<const float4 *>(rc + p * HD + gi * 8);
        const float4 *sp = reinterpret_cast<const float4 *>(rs + p * HD + gi * 8);
        const float4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
        const float c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        float x1[8], x2[8], y1[8], y2[8];
        unpack16<SWH_BF16>(*i1, x1);
        unpack16<SWH_BF16>(*i2, x2);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            if constexpr (!BWD) {
                y1[e] = round_bf16(x1[e] * c[e]) + round_bf16(-x2[e] * sn[e]);
                y2[e] = round_bf16(x2[e] * c[e]) + round_bf16(x1[e] * sn[e]);
            } else {  // x = dy here, y = dx
                y1[e] = round_bf16(x1[e] * c[e]) + round_bf16(x2[e] * sn[e]);
                y2[e] = round_bf16(x2[e] * c[e]) - round_bf16(x1[e] * sn[e]);
            }
        }
        uint32_t o1[4], o2[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            o1[e] = (uint32_t)f32_to_bf16_bits(y1[2 * e]) | ((uint32_t)f32_to_bf16_bits(y1[2 * e + 1]) << 16);
            o2[e] = (uint32_t)f32_to_bf16_bits(y2[2 * e]) | ((uint32_t)f32_to_bf16_bits(y2[2 * e + 1]) << 16);
        }
        *a1 = uint4{o1[0], o1[1], o1[2], o1[3]};
        *a2 = uint4{o2[0], o2[1], o2[2], o2[3]};
    }
}


// ---------------------------------------------------------------------------
// fp32 variants (reference-precision mode: an fp32 model, as transformers runs
// one loaded with torch_dtype=float32).  No intermediate rounding; the
// formulas are the fp32 modules': y = w * (s * rsqrt(mean(s^2) + eps)),
// silu(g) * u, x*cos + rotate_half(x)*sin.  One element per lane, one wave
// per row for the norms (16-B vectors are not needed at these sizes).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rmsnorm_fwd_f32_kernel(const float *__restrict__ x, const float *__restrict__ res,
                                                              float *__restrict__ res_out, const float *__restrict__ w,
                                                              int64_t rows, int64_t H, float eps, float *__restrict__ y,
                                                              float *__restrict__ rstd_out) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    float ss = 0.f;
    for (int64_t h = lane; h < H; h += 64) {
        float a = x[r * H + h];
        if (res) {
            a += res[r * H + h];
            if (res_out) res_out[r * H + h] = a;
        }
        ss = fmaf(a, a, ss);
    }
    ss = wave_sum(ss);
    const float rs = rsqrtf(ss / (float)H + eps);
    if (lane == 0 && rstd_out) rstd_out[r] = rs;
    for (int64_t h = lane; h < H; h += 64) {
        const float a = res ? x[r * H + h] + res[r * H + h] : x[r * H + h];
        y[r * H + h] = w[h] * (a * rs);
    }
}

// a workgroup = 4 waves over rows r0 .. r0 + rpb (a wave per row at a time);
// each wave keeps its dw column sums in its own LDS row, summed per block at the end
__global__ __launch_bounds__(256) void rmsnorm_bwd_f32_kernel(const float *__restrict__ x, const float *__restrict__ w,
                                                              const float *__restrict__ rstd, const float *__restrict__ dy,
                                                              int64_t rows, int64_t H, float *__restrict__ dx,
                                                              float *__restrict__ dw_part, int64_t rpb,
                                                              const float *__restrict__ dres) {
    extern __shared__ float dws[];  // [4][H]
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int64_t h = lane; h < H; h += 64) dws[wid * H + h] = 0.f;
    const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
    for (int64_t r = r0 + wid; r < r1; r += 4) {
        const float rs = rstd[r];
        float c = 0.f;
        for (int64_t h = lane; h < H; h += 64) c = fmaf(dy[r * H + h] * w[h], x[r * H + h] * rs, c);
        c = wave_sum(c) / (float)H;
        for (int64_t h = lane; h < H; h += 64) {
            const float n = x[r * H + h] * rs, g = dy[r * H + h];
            dws[wid * H + h] = fmaf(g, n, dws[wid * H + h]);
            float d = rs * (g * w[h] - n * c);
            if (dres) d += dres[r * H + h];
            dx[r * H + h] = d;
        }
    }
    __syncthreads();
    for (int64_t h = threadIdx.x; h < H; h += 256)
        dw_part[(int64_t)blockIdx.x * H + h] = ((dws[h] + dws[H + h]) + dws[2 * H + h]) + dws[3 * H + h];
}

__global__ __launch_bounds__(256) void silu_mul_f32_kernel(const float *__restrict__ gu, const float *__restrict__ dout,
                                                           int64_t rows, int64_t I, float *__restrict__ out) {
    const int64_t total = rows * I;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = idx / I, i = idx - r * I;
        const float g = gu[r * 2 * I + i], u = gu[r * 2 * I + I + i];
        const float sg = 1.f / (1.f + expf(-g));
        if (!dout) {
            out[idx] = (g * sg) * u;
        } else {  // out = d gu [rows, 2I]
            const float d = dout[idx];
            out[r * 2 * I + i] = (d * u) * (sg * (1.f + g * (1.f - sg)));
            out[r * 2 * I + I + i] = d * (g * sg);
        }
    }
}

template <bool BWD>
__global__ __launch_bounds__(256) void qkv_rope_f32_kernel(float *__restrict__ qkv, const int64_t *__restrict__ pos,
                                                           const float *__restrict__ rc, const float *__restrict__ rsn,
                                                           int64_t R, int L, int Hq, int Hkv, int D,
                                                           float *__restrict__ q, float *__restrict__ k,
                                                           float *__restrict__ v) {
    const int HD = D / 2, H3 = Hq + 2 * Hkv;
    const int64_t total = R * H3 * HD;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(idx % HD);
        const int h = (int)((idx / HD) % H3);
        const int64_t r = idx / ((int64_t)HD * H3);
        const int64_t b = r / L, l = r - b * L;
        float *src = qkv + r * (int64_t)H3 * D + (int64_t)h * D;
        float *dst;
        if (h < Hq) dst = q + ((b * Hq + h) * (int64_t)L + l) * D;
        else if (h < Hq + Hkv) dst = k + ((b * Hkv + (h - Hq)) * (int64_t)L + l) * D;
        else dst = v + ((b * Hkv + (h - Hq - Hkv)) * (int64_t)L + l) * D;
        float *o = BWD ? src : dst;
        const float *in = BWD ? dst : src;
        const float x1 = in[i], x2 = in[i + HD];
        if (h >= Hq + Hkv) {
            o[i] = x1;
            o[i + HD] = x2;
            continue;
        }
        const int64_t p = pos[r] < 0 ? 0 : pos[r];
        const float c = rc[p * HD + i], s = rsn[p * HD + i];
        if (!BWD) {
            o[i] = x1 * c + (-x2) * s;
            o[i + HD] = x2 * c + x1 * s;
        } else {
            o[i] = x1 * c + x2 * s;
            o[i + HD] = x2 * c - x1 * s;
        }
    }
}


// ---------------------------------------------------------------------------
// Embedding weight gradient without atomics (deterministic): token rows are
// visited in the order of the stably sorted ids.  Phase 1: each block of
// kEmbPiece sorted positions sums its pieces of id-runs into fp32 rows of the
// workspace (row = the piece's first sorted position).  Phase 2: the head of
// each run adds its pieces in sorted order (a run continues at the next block
// start) and folds the sum into the gradient row once:
// g[id] = round(g[id] + round(sum)) — torch's fp32-accumulating embedding
// backward followed by the AccumulateGrad add (tied lm-head gradient first).
// ---------------------------------------------------------------------------
constexpr int kEmbPiece = 32;

template <int DT>
__global__ __launch_bounds__(128) void embed_bwd_piece_kernel(const int64_t *__restrict__ sid,
                                                              const int64_t *__restrict__ order,
                                                              const typename Elem<DT>::T *__restrict__ dy, int64_t N,
                                                              int64_t H, float *__restrict__ ws) {
    constexpr int PV = kPerVec<DT>;
    const int64_t c0 = ((int64_t)blockIdx.y * 128 + threadIdx.x) * PV;
    if (c0 >= H) return;
    const int64_t b0 = (int64_t)blockIdx.x * kEmbPiece, b1 = min(N, b0 + kEmbPiece);
    float acc[PV];
#pragma unroll
    for (int k = 0; k < PV; ++k) acc[k] = 0.f;
    int64_t start = b0, cur = sid[b0];
    auto flush = [&](int64_t at) {
        float4 *o = reinterpret_cast<float4 *>(ws + at * H + c0);
#pragma unroll
        for (int k = 0; k < PV / 4; ++k) o[k] = float4{acc[4 * k], acc[4 * k + 1], acc[4 * k + 2], acc[4 * k + 3]};
    };
    for (int64_t p = b0; p < b1; ++p) {
        const int64_t id = sid[p];
        if (id != cur) {
            flush(start);
#pragma unroll
            for (int k = 0; k < PV; ++k) acc[k] = 0.f;
            start = p;
            cur = id;
        }
        float x[PV];
        unpack16<DT>(*reinterpret_cast<const uint4 *>(dy + order[p] * H + c0), x);
#pragma unroll
        for (int k = 0; k < PV; ++k) acc[k] += x[k];
    }
    flush(start);
}

template <int DT>
__global__ __launch_bounds__(128) void embed_bwd_sum_kernel(const int64_t *__restrict__ sid, int64_t N, int64_t H,
                                                            int64_t V, const float *__restrict__ ws,
                                                            typename Elem<DT>::T *__restrict__ g) {
    constexpr int PV = kPerVec<DT>;
    const int64_t p = blockIdx.x;
    const int64_t id = sid[p];
    if ((p > 0 && sid[p - 1] == id) || id < 0 || id >= V) return;  // not a run head
    const int64_t c0 = ((int64_t)blockIdx.y * 128 + threadIdx.x) * PV;
    if (c0 >= H) return;
    float tot[PV];
#pragma unroll
    for (int k = 0; k < PV; ++k) tot[k] = ws[p * H + c0 + k];
    for (int64_t q = (p / kEmbPiece + 1) * kEmbPiece; q < N && sid[q] == id; q += kEmbPiece) {
#pragma unroll
        for (int k = 0; k < PV; ++k) tot[k] += ws[q * H + c0 + k];
    }
    if constexpr (DT == SWH_F32) {
#pragma unroll
        for (int k = 0; k < PV; ++k) g[id * H + c0 + k] += tot[k];
    } else {
        float cur[PV];
        uint4 *gp = reinterpret_cast<uint4 *>(g + id * H + c0);
        unpack16<DT>(*gp, cur);
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = (uint32_t)f32_to_bf16_bits(cur[2 * k] + round_bf16(tot[2 * k])) |
                   ((uint32_t)f32_to_bf16_bits(cur[2 * k + 1] + round_bf16(tot[2 * k + 1])) << 16);
        *gp = uint4{o[0], o[1], o[2], o[3]};
    }
}


// ---------------------------------------------------------------------------
// Column sums of a tall [rows, cols] matrix (the bias gradient: sum over tokens
// of dy), deterministic: a workgroup sums one chunk of rows for 512 (bf16) /
// 256 (f32) columns, its 4 waves taking every 4th row, then adds the waves in
// fixed order into one fp32 partial row per chunk; swh_rmsnorm_dw_accum folds
// the partial rows into the gradient view.
// ---------------------------------------------------------------------------
template <int DT>
__global__ __launch_bounds__(256) void colsum_partials_kernel(const typename Elem<DT>::T *__restrict__ x, int64_t rows,
                                                              int64_t cols, int64_t rpc, float *__restrict__ part) {
    constexpr int PV = kPerVec<DT>;
    __shared__ float red[4][64 * PV];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t c0 = ((int64_t)blockIdx.x * 64 + lane) * PV;
    const int64_t r0 = (int64_t)blockIdx.y * rpc, r1 = min(rows, r0 + rpc);
    float acc[PV];
#pragma unroll
    for (int k = 0; k < PV; ++k) acc[k] = 0.f;
    if (c0 < cols) {
        int64_t r = r0 + wid;
        for (; r + 12 < r1; r += 16) {  // four rows' loads in flight
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4 *>(x + (r + 4 * u) * cols + c0);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float f[PV];
                unpack16<DT>(v[u], f);
#pragma unroll
                for (int k = 0; k < PV; ++k) acc[k] += f[k];
            }
        }
        for (; r < r1; r += 4) {
            float f[PV];
            unpack16<DT>(*reinterpret_cast<const uint4 *>(x + r * cols + c0), f);
#pragma unroll
            for (int k = 0; k < PV; ++k) acc[k] += f[k];
        }
    }
#pragma unroll
    for (int k = 0; k < PV; ++k) red[wid][lane * PV + k] = acc[k];
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * PV; i += 256) {
        const int64_t c = (int64_t)blockIdx.x * 64 * PV + i;
        if (c < cols) part[(int64_t)blockIdx.y * cols + c] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
    }
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int swh_rmsnorm_fwd(const void *x, const void *residual, void *residual_out, const void *weight,
                               int64_t rows, int64_t H, float eps, void *y, float *rstd, int32_t dtype, void *stream) {
    if (!x || !weight || !y || rows < 0 || H <= 0 || H % 8) return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F32) return SWH_E_DTYPE;
    if (rows == 0) return SWH_OK;
    if (dtype == SWH_F32) {
        rmsnorm_fwd_f32_kernel<<<dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(
            static_cast<const float *>(x), static_cast<const float *>(residual), static_cast<float *>(residual_out),
            static_cast<const float *>(weight), rows, H, eps, static_cast<float *>(y), rstd);
        return launch_status();
    }
    rmsnorm_fwd_kernel<<<dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(x), static_cast<const uint16_t *>(residual), static_cast<uint16_t *>(residual_out),
        static_cast<const uint16_t *>(weight), rows, H, eps, static_cast<uint16_t *>(y), rstd);
    return launch_status();
}

// d weight: gw[h] = bf16(gw[h] + bf16(sum_b part[b][h])) — the partial column sums of
// swh_rmsnorm_bwd folded into the bf16 gradient view.  A workgroup = 64 columns x 4 row
// slices: slice s sums partial rows s, s + 4, ... of its range (loads issued 8 at a time),
// then the 4 slice sums add in fixed order through LDS.  Long column sums (the 544
// partial rows of a 17408-token pass would leave H / 64 = 14 workgroups streaming 2 MB)
// go in two stages: stage 1 splits the rows into ranges of `rps`, each range summed by
// its own workgroup into the range's first row (read by no other workgroup); stage 2
// sums those rows (stride rps) and folds them in.  Fixed order throughout.
constexpr int kDwSlices = 4;       // 256-thread workgroups: they fit beside the GEMMs they overlap
constexpr int kDwRangeRows = 32;  // stage-1 rows per range
template <int DT, bool FOLD>
__global__ __launch_bounds__(64 * kDwSlices) void rmsnorm_dw_accum_kernel(float *__restrict__ part, int64_t nb,
                                                                         int64_t H, int64_t stride,
                                                                         typename Elem<DT>::T *__restrict__ gw) {
    __shared__ float red[kDwSlices][64];
    const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
    const int64_t h = (int64_t)blockIdx.x * 64 + c;
    const int64_t r0 = FOLD ? 0 : (int64_t)blockIdx.y * kDwRangeRows;  // stage 1: this workgroup's range
    const int64_t r1 = FOLD ? nb : min(nb, r0 + kDwRangeRows);
    float t = 0.f;
    if (h < H) {
        int64_t b = r0 + sl;
        for (; b + 7 * kDwSlices < r1; b += 8 * kDwSlices) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = part[(b + j * kDwSlices) * stride * H + h];
#pragma unroll
            for (int j = 0; j < 8; ++j) t += v[j];
        }
        for (; b < r1; b += kDwSlices) t += part[b * stride * H + h];
    }
    red[sl][c] = t;
    __syncthreads();
    if (sl == 0 && h < H) {
        float u = 0.f;
#pragma unroll
        for (int q = 0; q < kDwSlices; ++q) u += red[q][c];
        if constexpr (!FOLD) part[r0 * H + h] = u;
        else if constexpr (DT == SWH_F32) gw[h] += u;
        else gw[h] = f32_to_bf16_bits(bf16_bits_to_f32(gw[h]) + round_bf16(u));
    }
}

template <int DT>
int dw_accum(float *part, int64_t nb, int64_t H, typename Elem<DT>::T *gw, hipStream_t st) {
    const unsigned cb = (unsigned)((H + 63) / 64);
    if (nb <= 2 * kDwRangeRows) {
        rmsnorm_dw_accum_kernel<DT, true><<<dim3(cb), 64 * kDwSlices, 0, st>>>(part, nb, H, 1, gw);
        return launch_status();
    }
    const int64_t nr = (nb + kDwRangeRows - 1) / kDwRangeRows;
    rmsnorm_dw_accum_kernel<DT, false><<<dim3(cb, (unsigned)nr), 64 * kDwSlices, 0, st>>>(part, nb, H, 1, gw);
    rmsnorm_dw_accum_kernel<DT, true><<<dim3(cb), 64 * kDwSlices, 0, st>>>(part, nr, H, kDwRangeRows, gw);
    return launch_status();
}

extern "C" int swh_rmsnorm_dw_accum(const float *dw_partial, int64_t nblocks, int64_t H, void *grad_w, int32_t dtype,
                                    void *stream) {
    if (!dw_partial || !grad_w || nblocks <= 0 || H <= 0) return SWH_E_ARG;
    hipStream_t st = static_cast<hipStream_t>(stream);
    float *part = const_cast<float *>(dw_partial);  // stage 1 writes each range's sum into its first row
    if (dtype == SWH_BF16) return dw_accum<SWH_BF16>(part, nblocks, H, static_cast<uint16_t *>(grad_w), st);
    if (dtype == SWH_F32) return dw_accum<SWH_F32>(part, nblocks, H, static_cast<float *>(grad_w), st);
    return SWH_E_DTYPE;
}

extern "C" int swh_rmsnorm_bwd(const void *x, const void *weight, const float *rstd, const void *dy, int64_t rows,
                               int64_t H, void *dx, float *dw_partial, int64_t rows_per_block, const void *dres,
                               int32_t dtype, void *stream) {
    if (!x || !weight || !rstd || !dy || !dx || !dw_partial || rows < 0 || H <= 0 || H % 8 ||
        H > 64 * 8 * kNormBwdVec || rows_per_block <= 0 || rows_per_block > 4096)
        return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F32) return SWH_E_DTYPE;
    if (rows == 0) return SWH_OK;
    const unsigned nb = (unsigned)((rows + rows_per_block - 1) / rows_per_block);
    if (dtype == SWH_F32) {
        rmsnorm_bwd_f32_kernel<<<dim3(nb), dim3(256), 4 * H * sizeof(float), static_cast<hipStream_t>(stream)>>>(
            static_cast<const float *>(x), static_cast<const float *>(weight), rstd, static_cast<const float *>(dy),
            rows, H, static_cast<float *>(dx), dw_partial, rows_per_block, static_cast<const float *>(dres));
        return launch_status();
    }
    const size_t lds = (kNormBwdThreads / 64) * H * sizeof(float);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const auto *X = static_cast<const uint16_t *>(x), *Wt = static_cast<const uint16_t *>(weight);
    const auto *DY = static_cast<const uint16_t *>(dy);
    auto *DX = static_cast<uint16_t *>(dx);
#define SWH_NORM_BWD(V) \
    rmsnorm_bwd_kernel<V><<<dim3(nb), dim3(kNormBwdThreads), lds, st>>>(X, Wt, rstd, DY, rows, H, DX, dw_partial, \
                                                                        rows_per_block, static_cast<const uint16_t *>(dres))
    if (H <= 64 * 8 * 2) SWH_NORM_BWD(2);
    else if (H <= 64 * 8 * 4) SWH_NORM_BWD(4);
    else SWH_NORM_BWD(8);
#undef SWH_NORM_BWD
    return launch_status();
}

static unsigned ew_grid(int64_t work) {
    int64_t g = (work + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;
    return (unsigned)(g < 1 ? 1 : g);
}

extern "C" int swh_silu_mul_fwd(const void *gu, int64_t rows, int64_t I, void *out, int32_t dtype, void *stream) {
    if (!gu || !out || rows < 0 || I <= 0 || I % 8) return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F32) return SWH_E_DTYPE;
    if (rows == 0) return SWH_OK;
    if (dtype == SWH_F32) {
        silu_mul_f32_kernel<<<ew_grid(rows * I), 256, 0, static_cast<hipStream_t>(stream)>>>(
            static_cast<const float *>(gu), nullptr, rows, I, static_cast<float *>(out));
        return launch_status();
    }
    silu_mul_fwd_kernel<<<ew_grid(rows * I / 8), 256, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(gu), rows, I, static_cast<uint16_t *>(out));
    return launch_status();
}

extern "C" int swh_silu_mul_bwd(const void *gu, const void *dout, int64_t rows, int64_t I, void *dgu, int32_t dtype,
                                void *stream) {
    if (!gu || !dout || !dgu || rows < 0 || I <= 0 || I % 8) return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F32) return SWH_E_DTYPE;
    if (rows == 0) return SWH_OK;
    if (dtype == SWH_F32) {
        silu_mul_f32_kernel<<<ew_grid(rows * I), 256, 0, static_cast<hipStream_t>(stream)>>>(
            static_cast<const float *>(gu), static_cast<const float *>(dout), rows, I, static_cast<float *>(dgu));
        return launch_status();
    }
    silu_mul_bwd_kernel<<<ew_grid(rows * I / 8), 256, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(gu), static_cast<const uint16_t *>(dout), rows, I, static_cast<uint16_t *>(dgu));
    return launch_status();
}

extern "C" int swh_fold_norm(const void *jobs, int32_t njobs, int64_t total_rows, void *stream) {
    if (!jobs || njobs <= 0 || njobs > kFoldMaxJobs || total_rows <= 0) return SWH_E_ARG;
    const int64_t nchunk = (total_rows + kFoldRows - 1) / kFoldRows;
    const int64_t grid = nchunk < 4096 ? nchunk : 4096;
    fold_norm_kernel<<<dim3((unsigned)grid), 256, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const FoldJob *>(jobs), njobs, total_rows);
    return launch_status();
}

extern "C" int swh_embed_gather(const void *table, const int64_t *ids, int64_t B, int64_t H, void *x, float *ss_out,
                                void *stream) {
    if (!table || !ids || !x || B < 0 || H <= 0 || H % 16) return SWH_E_ARG;
    if (B == 0) return SWH_OK;
    embed_gather_kernel<<<dim3((unsigned)B), 128, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t *>(table), ids, H, static_cast<uint16_t *>(x), ss_out);
    return launch_status();
}

extern "C" int swh_qkv_rope(void *qkv, const int64_t *positions, const float *rope_cos, const float *rope_sin,
                            int64_t B, int64_t L, int32_t Hq, int32_t Hkv, int32_t D, void *q, void *k, void *v,
                            int32_t backward, int32_t dtype, void *stream) {
    if (!qkv || !positions || !rope_cos || !rope_sin || !q || !k || !v || B < 0 || L < 0 || Hq <= 0 || Hkv <= 0 ||
        D <= 0 || D % 16)
        return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F32) return SWH_E_DTYPE;
    const int64_t R = B * L;
    if (R == 0) return SWH_OK;
    if (dtype == SWH_F32) {
        int64_t g = (R * (Hq + 2 * Hkv) * (D / 2) + 255) / 256;
        if (g > 256 * 32) g = 256 * 32;
        auto *Qf = static_cast<float *>(q), *Kf = static_cast<float *>(k), *Vf = static_cast<float *>(v);
        auto *X = static_cast<float *>(qkv);
        if (backward)
            qkv_rope_f32_kernel<true><<<dim3((unsigned)g), 256, 0, static_cast<hipStream_t>(stream)>>>(
                X, positions, rope_cos, rope_sin, R, (int)L, Hq, Hkv, D, Qf, Kf, Vf);
        else
            qkv_rope_f32_kernel<false><<<dim3((unsigned)g), 256, 0, static_cast<hipStream_t>(stream)>>>(
                X, positions, rope_cos, rope_sin, R, (int)L, Hq, Hkv, D, Qf, Kf, Vf);
        return launch_status();
    }
    const int64_t work = R * (Hq + 2 * Hkv) * (D / 16);
    int64_t grid = (work + 255) / 256;
    if (grid > 256 * 32) grid = 256 * 32;
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto *Q = static_cast<uint16_t *>(q), *K = static_cast<uint16_t *>(k), *V = static_cast<uint16_t *>(v);
    if (backward)
        qkv_rope_kernel<true><<<dim3((unsigned)grid), 256, 0, s>>>(static_cast<uint16_t *>(qkv), positions, rope_cos,
                                                                  rope_sin, R, (int)L, Hq, Hkv, D, Q, K, V);
    else
        qkv_rope_kernel<false><<<dim3((unsigned)grid), 256, 0, s>>>(static_cast<uint16_t *>(qkv), positions, rope_cos,
                                                                   rope_sin, R, (int)L, Hq, Hkv, D, Q, K, V);
    return launch_status();
}

extern "C" int64_t swh_embedding_bwd_workspace_bytes(int64_t N, int64_t H) { return N * H * (int64_t)sizeof(float); }

extern "C" int swh_embedding_bwd(const int64_t *sorted_ids, const int64_t *order, const void *dy, int64_t N, int64_t H,
                                 int64_t V, void *grad_table, int32_t dtype, float *workspace, void *stream) {
    if (!sorted_ids || !order || !dy || !grad_table || !workspace || N < 0 || H <= 0 || V <= 0) return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F32) return SWH_E_DTYPE;
    const int pv = dtype == SWH_F32 ? 4 : 8;
    if (H % pv) return SWH_E_ARG;
    if (N == 0) return SWH_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const unsigned gy = (unsigned)((H / pv + 127) / 128);
    const dim3 g1((unsigned)((N + kEmbPiece - 1) / kEmbPiece), gy), g2((unsigned)N, gy);
    if (dtype == SWH_BF16) {
        embed_bwd_piece_kernel<SWH_BF16><<<g1, 128, 0, st>>>(sorted_ids, order, static_cast<const uint16_t *>(dy), N, H,
                                                             workspace);
        embed_bwd_sum_kernel<SWH_BF16><<<g2, 128, 0, st>>>(sorted_ids, N, H, V, workspace,
                                                           static_cast<uint16_t *>(grad_table));
    } else {
        embed_bwd_piece_kernel<SWH_F32><<<g1, 128, 0, st>>>(sorted_ids, order, static_cast<const float *>(dy), N, H,
                                                            workspace);
        embed_bwd_sum_kernel<SWH_F32><<<g2, 128, 0, st>>>(sorted_ids, N, H, V, workspace,
                                                          static_cast<float *>(grad_table));
    }
    return launch_status();
}

extern "C" int swh_colsum_partials(const void *x, int64_t rows, int64_t cols, int64_t rows_per_chunk, float *part,
                                   int32_t dtype, void *stream) {
    if (!x || !part || rows < 0 || cols <= 0 || rows_per_chunk <= 0) return SWH_E_ARG;
    if (dtype != SWH_BF16 && dtype != SWH_F32) return SWH_E_DTYPE;
    const int pv = dtype == SWH_F32 ? 4 : 8;
    if (cols % pv || (reinterpret_cast<uintptr_t>(x) & 15)) return SWH_E_ARG;
    if (rows == 0) return SWH_OK;
    const dim3 grid((unsigned)((cols / pv + 63) / 64), (unsigned)((rows + rows_per_chunk - 1) / rows_per_chunk));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (dtype == SWH_BF16)
        colsum_partials_kernel<SWH_BF16><<<grid, 256, 0, st>>>(static_cast<const uint16_t *>(x), rows, cols,
                                                               rows_per_chunk, part);
    else
        colsum_partials_kernel<SWH_F32><<<grid, 256, 0, st>>>(static_cast<const float *>(x), rows, cols,
                                                              rows_per_chunk, part);
    return launch_status();
}
