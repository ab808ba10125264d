// Decode-step kernels of the rollout engine (batch <= 64 rows per tile):
//
//  * swh_decode_gemm — weight-streaming "skinny" GEMM  Y[M,N] = X[M,K] W[N,K]^T
//    on MFMA v_mfma_f32_16x16x32_bf16, with the decoder's neighbours fused:
//      prologue  RMSNorm of X (Qwen2RMSNorm rounding points)      [qkv, gate_up, lm head]
//      epilogue  + bias                                           [qkv]
//                residual: s = bf16(s + bf16(acc)) in place       [o_proj, down_proj]
//                SiLU gate: y = bf16(bf16(silu(bf16 g)) * bf16 u) [gate_up]
//    One workgroup = all M rows x NB output columns; its 4 waves split K four
//    ways and meet in LDS.  W (the only HBM stream) is read exactly once,
//    16 B per lane, two k-steps unrolled so every 128-B line is consumed by one
//    wave; X is tiny and L2-resident.  Grid = N / NB workgroups.
//    Replaces the hipBLASLt M=64 GEMMs (measured 0.6 TB/s) plus the separate
//    RMSNorm / SiLU / residual launches of the decode layer.
//
//  * attention decode (GQA) — one workgroup (8 waves) per (kv head, sequence):
//    RoPE + KV append, scores with D/8 lanes per key (16-B K loads, coalesced
//    rows), softmax in LDS, P·V with the same lane map, shuffle + LDS merge.
#include "common.hpp"

namespace swh {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kGemmThreads = 256;
constexpr int kRows = 64;  // rows per workgroup tile (M tile)

enum : int { EPI_PLAIN = 0, EPI_RESIDUAL = 1, EPI_SILU = 2 };

__device__ __forceinline__ bf16x8 as_bf16x8(const uint4 &v) { return __builtin_bit_cast(bf16x8, v); }

// A fragment of normalised X: bf16(w * bf16(x * rstd)) for 8 consecutive k.
__device__ __forceinline__ uint4 norm_frag(const uint4 &xv, const uint4 &wv, float rs) {
    float x[8], w[8];
    unpack16<SWH_BF16>(xv, x);
    unpack16<SWH_BF16>(wv, w);
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float a = w[2 * k] * round_bf16(x[2 * k] * rs);
        const float b = w[2 * k + 1] * round_bf16(x[2 * k + 1] * rs);
        o[k] = (uint32_t)f32_to_bf16_bits(a) | ((uint32_t)f32_to_bf16_bits(b) << 16);
    }
    return uint4{o[0], o[1], o[2], o[3]};
}

// NB = output columns per workgroup (multiple of 16); CB = NB / 16 column blocks.
template <int NB, bool NORM, int EPI, bool BIAS>
__global__ __launch_bounds__(kGemmThreads) void decode_gemm_kernel(
    const uint16_t *__restrict__ x, const uint16_t *__restrict__ w, int M, int N, int K,
    const uint16_t *__restrict__ norm_w, float eps, const uint16_t *__restrict__ bias, uint16_t *__restrict__ res,
    uint16_t *__restrict__ y, int ldy) {
    constexpr int CB = NB / 16;
    __shared__ float rstd_s[kRows];
    __shared__ float part[4][kRows][NB + 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int m0 = blockIdx.y * kRows;
    const int n0 = blockIdx.x * (EPI == EPI_SILU ? NB / 2 : NB);

    // ---- prologue: per-row rstd of X (fused RMSNorm)
    if constexpr (NORM) {
        for (int rr = wid; rr < kRows; rr += 4) {
            const int r = min(m0 + rr, M - 1);
            const uint4 *xr = reinterpret_cast<const uint4 *>(x + (int64_t)r * K);
            float ss = 0.f;
            for (int v = lane; v < K / 8; v += 64) {
                float a[8];
                unpack16<SWH_BF16>(xr[v], a);
#pragma unroll
                for (int k = 0; k < 8; ++k) ss = fmaf(a[k], a[k], ss);
            }
            ss = wave_sum(ss);
            if (lane == 0) rstd_s[rr] = rsqrtf(ss / (float)K + eps);
        }
        __syncthreads();
    }

    // ---- main loop: wave `wid` owns k in [kb, ke)
    const int kw = K / 4;
    const int kb = wid * kw, ke = kb + kw;
    const int rl = lane & 15, kq = (lane >> 4) * 8;  // fragment row/col within 16, k offset within 32
    f32x4 acc[4][CB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const uint16_t *xrow[4];
    float rs[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = min(m0 + i * 16 + rl, M - 1);
        xrow[i] = x + (int64_t)r * K;
        rs[i] = NORM ? rstd_s[i * 16 + rl] : 1.f;
    }
    const uint16_t *wrow[CB];
#pragma unroll
    for (int j = 0; j < CB; ++j) {
        int n;
        if constexpr (EPI == EPI_SILU) {
            // column block j: first 8 columns gate rows, last 8 the matching up rows
            const int c = j * 8 + (rl & 7);
            n = (rl < 8) ? n0 + c : N + n0 + c;
        } else {
            n = n0 + j * 16 + rl;
        }
        wrow[j] = w + (int64_t)n * K;
    }

#pragma unroll 2
    for (int k0 = kb; k0 < ke; k0 += 32) {
        const int k = k0 + kq;
        uint4 bv[CB];
#pragma unroll
        for (int j = 0; j < CB; ++j) bv[j] = ld_nt(reinterpret_cast<const uint4 *>(wrow[j] + k));
        uint4 av[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = *reinterpret_cast<const uint4 *>(xrow[i] + k);
        if constexpr (NORM) {
            const uint4 nw = *reinterpret_cast<const uint4 *>(norm_w + k);
#pragma unroll
            for (int i = 0; i < 4; ++i) av[i] = norm_frag(av[i], nw, rs[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < CB; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(av[i]), as_bf16x8(bv[j]), acc[i][j],
                                                                    0, 0, 0);
    }

    // ---- cross-wave split-K merge in LDS
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) part[wid][i * 16 + (lane >> 4) * 4 + e][j * 16 + rl] = acc[i][j][e];
    __syncthreads();

    // ---- epilogue
    if constexpr (EPI == EPI_SILU) {
        constexpr int NO = NB / 2;  // output columns of this tile
        for (int idx = threadIdx.x; idx < kRows * NO; idx += kGemmThreads) {
            const int r = idx / NO, c = idx - r * NO;
            const int gr = m0 + r;
            if (gr >= M) continue;
            const int jb = c / 8, cc = c - jb * 8;
            const int cg = jb * 16 + cc, cu = cg + 8;
            float g = 0.f, u = 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                g += part[q][r][cg];
                u += part[q][r][cu];
            }
            g = round_bf16(g);
            u = round_bf16(u);
            const float a = round_bf16(g / (1.f + expf(-g))) * u;
            y[(int64_t)gr * ldy + n0 + c] = f32_to_bf16_bits(a);
        }
    } else {
        for (int idx = threadIdx.x; idx < kRows * NB; idx += kGemmThreads) {
            const int r = idx / NB, c = idx - r * NB;
            const int gr = m0 + r, gc = n0 + c;
            if (gr >= M || gc >= N) continue;
            float v = part[0][r][c] + part[1][r][c] + part[2][r][c] + part[3][r][c];
            if constexpr (BIAS) v += bf16_bits_to_f32(bias[gc]);
            if constexpr (EPI == EPI_RESIDUAL) {
                uint16_t *s = res + (int64_t)gr * ldy + gc;
                *s = f32_to_bf16_bits(bf16_bits_to_f32(*s) + round_bf16(v));
            } else {
                y[(int64_t)gr * ldy + gc] = f32_to_bf16_bits(v);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Attention decode (GQA): one workgroup of 8 waves per (kv head, sequence).
// ---------------------------------------------------------------------------
constexpr int kAttnThreads = 512;
constexpr int kAttnWaves = kAttnThreads / 64;

template <int D, int GQ>
__global__ __launch_bounds__(kAttnThreads) void attn_decode_kernel(
    const uint16_t *__restrict__ qkv, uint16_t *__restrict__ kc, uint16_t *__restrict__ vc,
    const float *__restrict__ rcos, const float *__restrict__ rsin, const int32_t *__restrict__ plen,
    const int32_t *__restrict__ state, int Hq, int Hkv, int Tmax, float scale, uint16_t *__restrict__ out) {
    constexpr int LPK = D / 8;     // lanes per key row (8 dims each, one 16-B load)
    constexpr int KPW = 64 / LPK;  // keys per wave per iteration
    constexpr int HD = D / 2;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *q_s = smem;                                  // [GQ][D]
    float *red = q_s + GQ * D;                          // [waves][GQ][D]
    float *stat = red + kAttnWaves * GQ * D;            // m[GQ], l[GQ]
    uint16_t *knew = reinterpret_cast<uint16_t *>(stat + 2 * GQ);  // [D]
    uint16_t *vnew = knew + D;                          // [D]
    float *sc = reinterpret_cast<float *>(vnew + D);    // [GQ][n]  (16-B aligned: D multiple of 8)

    const int kvh = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // state[0] = index of the token sampled this step; the input token is state[0] - 1
    const int step = state[0] - 1, P = state[1];
    const int pl = plen[b];
    const int slot_new = P + step;
    const int start = P - pl;
    const int pos = pl + step;
    uint16_t *ob = out + b * (int64_t)Hq * D + kvh * GQ * D;
    if (step < 0 || slot_new >= Tmax || pl < 0 || pl > P) {  // never write outside the cache
        for (int idx = tid; idx < GQ * D; idx += kAttnThreads) ob[idx] = 0x7fc0;  // NaN: fail loudly
        return;
    }
    const int n = slot_new - start + 1;  // keys incl. the new one
    const uint16_t *row = qkv + b * (int64_t)(Hq + 2 * Hkv) * D;
    const int64_t cbase = (b * Hkv + kvh) * (int64_t)Tmax * D;

    for (int idx = tid; idx < (GQ + 1) * HD; idx += kAttnThreads) {
        const int hh = idx / HD, i = idx - hh * HD;
        const float c = rcos[(int64_t)pos * HD + i], s = rsin[(int64_t)pos * HD + i];
        const uint16_t *src = (hh < GQ) ? row + (kvh * GQ + hh) * D : row + (Hq + kvh) * D;
        const float x1 = bf16_bits_to_f32(src[i]), x2 = bf16_bits_to_f32(src[i + HD]);
        const float o1 = round_bf16(round_bf16(x1 * c) + round_bf16(-x2 * s));
        const float o2 = round_bf16(round_bf16(x2 * c) + round_bf16(x1 * s));
        if (hh < GQ) {
            q_s[hh * D + i] = o1;
            q_s[hh * D + i + HD] = o2;
        } else {
            knew[i] = f32_to_bf16_bits(o1);
            knew[i + HD] = f32_to_bf16_bits(o2);
        }
    }
    for (int d = tid; d < D; d += kAttnThreads) vnew[d] = row[(Hq + Hkv + kvh) * D + d];
    __syncthreads();
    for (int d = tid; d < D; d += kAttnThreads) {
        kc[cbase + (int64_t)slot_new * D + d] = knew[d];
        vc[cbase + (int64_t)slot_new * D + d] = vnew[d];
    }

    const int part_ = lane % LPK, kin = lane / LPK;
    float qreg[GQ][8];
#pragma unroll
    for (int h = 0; h < GQ; ++h)
#pragma unroll
        for (int k = 0; k < 8; ++k) qreg[h][k] = q_s[h * D + part_ * 8 + k];

    // ---- pass 1: scores
    const uint16_t *kb_ = kc + cbase + (int64_t)start * D + part_ * 8;
    for (int kk = wid * KPW + kin; kk < n; kk += kAttnWaves * KPW) {
        float kv[8];
        if (kk == n - 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) kv[k] = bf16_bits_to_f32(knew[part_ * 8 + k]);
        } else {
            unpack16<SWH_BF16>(*reinterpret_cast<const uint4 *>(kb_ + (int64_t)kk * D), kv);
        }
        float dot[GQ];
#pragma unroll
        for (int h = 0; h < GQ; ++h) {
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) s = fmaf(qreg[h][k], kv[k], s);
#pragma unroll
            for (int o = 1; o < LPK; o <<= 1) s += __shfl_xor(s, o, kWave);
            dot[h] = s;
        }
        if (part_ == 0) {
#pragma unroll
            for (int h = 0; h < GQ; ++h) sc[h * n + kk] = dot[h] * scale;
        }
    }
    __syncthreads();
    // ---- softmax per head (one wave per head)
    for (int h = wid; h < GQ; h += kAttnWaves) {
        float mx = kNegInf;
        for (int k = lane; k < n; k += 64) mx = fmaxf(mx, sc[h * n + k]);
        mx = wave_max(mx);
        float sum = 0.f;
        for (int k = lane; k < n; k += 64) {
            const float p = expf(sc[h * n + k] - mx);
            sc[h * n + k] = p;
            sum += p;
        }
        sum = wave_sum(sum);
        if (lane == 0) stat[GQ + h] = sum;
    }
    __syncthreads();
    // ---- pass 2: P V with the same lane map
    float acc[GQ][8];
#pragma unroll
    for (int h = 0; h < GQ; ++h)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[h][k] = 0.f;
    const uint16_t *vb_ = vc + cbase + (int64_t)start * D + part_ * 8;
    for (int kk = wid * KPW + kin; kk < n; kk += kAttnWaves * KPW) {
        float vv[8];
        if (kk == n - 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) vv[k] = bf16_bits_to_f32(vnew[part_ * 8 + k]);
        } else {
            unpack16<SWH_BF16>(*reinterpret_cast<const uint4 *>(vb_ + (int64_t)kk * D), vv);
        }
#pragma unroll
        for (int h = 0; h < GQ; ++h) {
            const float p = sc[h * n + kk];
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[h][k] = fmaf(p, vv[k], acc[h][k]);
        }
    }
    // merge the KPW key groups of the wave (lanes differing in the kin bits)
#pragma unroll
    for (int h = 0; h < GQ; ++h)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float v = acc[h][k];
#pragma unroll
            for (int o = LPK; o < 64; o <<= 1) v += __shfl_xor(v, o, kWave);
            acc[h][k] = v;
        }
    if (kin == 0) {
#pragma unroll
        for (int h = 0; h < GQ; ++h)
#pragma unroll
            for (int k = 0; k < 8; ++k) red[(wid * GQ + h) * D + part_ * 8 + k] = acc[h][k];
    }
    __syncthreads();
    for (int idx = tid; idx < GQ * D; idx += kAttnThreads) {
        const int h = idx / D;
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < kAttnWaves; ++q) v += red[q * GQ * D + idx];
        ob[idx] = f32_to_bf16_bits(v / stat[GQ + h]);
    }
}

template <int D, int GQ>
int launch_attn(const uint16_t *q, uint16_t *kc, uint16_t *vc, const float *rc, const float *rs, const int32_t *pl,
                const int32_t *st, int64_t B, int Hq, int Hkv, int Tmax, float scale, uint16_t *o, hipStream_t s) {
    const size_t lds = sizeof(float) * (GQ * D + kAttnWaves * GQ * D + 2 * GQ) + 2 * D * sizeof(uint16_t) +
                       sizeof(float) * (size_t)GQ * Tmax;
    if (lds > 160 * 1024) return SWH_E_ARG;
    attn_decode_kernel<D, GQ><<<dim3((unsigned)Hkv, (unsigned)B), kAttnThreads, lds, s>>>(q, kc, vc, rc, rs, pl, st,
                                                                                         Hq, Hkv, Tmax, scale, o);
    return launch_status();
}

template <int D>
int attn_dispatch_gq(int gq, const uint16_t *q, uint16_t *kc, uint16_t *vc, const float *rc, const float *rs,
                     const int32_t *pl, const int32_t *st, int64_t B, int Hq, int Hkv, int Tmax, float scale,
                     uint16_t *o, hipStream_t s) {
    switch (gq) {
    case 1: return launch_attn<D, 1>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 2: return launch_attn<D, 2>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 3: return launch_attn<D, 3>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 4: return launch_attn<D, 4>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 5: return launch_attn<D, 5>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 6: return launch_attn<D, 6>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 7: return launch_attn<D, 7>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    case 8: return launch_attn<D, 8>(q, kc, vc, rc, rs, pl, st, B, Hq, Hkv, Tmax, scale, o, s);
    default: return SWH_E_ARG;
    }
}

}  // namespace
}  // namespace swh

using namespace swh;

extern "C" int swh_attn_decode(const void *qkv, void *k_cache, void *v_cache, const float *rope_cos,
                               const float *rope_sin, const int32_t *prompt_len, const int32_t *state, int64_t B,
                               int32_t Hq, int32_t Hkv, int32_t D, int32_t Tmax, float scale, void *out,
                               void *stream) {
    if (!qkv || !k_cache || !v_cache || !rope_cos || !rope_sin || !prompt_len || !state || !out || B < 0 || Hkv <= 0 ||
        Hq % Hkv || Tmax <= 0)
        return SWH_E_ARG;
    if (B == 0) return SWH_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const auto *q = static_cast<const uint16_t *>(qkv);
    auto *kc = static_cast<uint16_t *>(k_cache), *vc = static_cast<uint16_t *>(v_cache);
    auto *o = static_cast<uint16_t *>(out);
    const int gq = Hq / Hkv;
    if (D == 64) return attn_dispatch_gq<64>(gq, q, kc, vc, rope_cos, rope_sin, prompt_len, state, B, Hq, Hkv, Tmax, scale, o, s);
    if (D == 128) return attn_dispatch_gq<128>(gq, q, kc, vc, rope_cos, rope_sin, prompt_len, state, B, Hq, Hkv, Tmax, scale, o, s);
    return SWH_E_ARG;
}

extern "C" int swh_decode_gemm(const void *x, const void *w, int64_t M, int64_t N, int64_t K, const void *norm_w,
                               float eps, const void *bias, void *residual, int32_t silu, void *y, int64_t ldy,
                               void *stream) {
    if (!x || !w || M <= 0 || N <= 0 || K <= 0 || K % 128 || M > (1 << 20) || N >= (1 << 30) || K >= (1 << 30))
        return SWH_E_ARG;
    if (residual && (silu || bias)) return SWH_E_ARG;
    if (!residual && !y) return SWH_E_ARG;
    if (((uintptr_t)x | (uintptr_t)w) & 15) return SWH_E_ARG;
    if (norm_w && ((uintptr_t)norm_w & 15)) return SWH_E_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const auto *X = static_cast<const uint16_t *>(x);
    const auto *W = static_cast<const uint16_t *>(w);
    const auto *NW = static_cast<const uint16_t *>(norm_w);
    const auto *Bs = static_cast<const uint16_t *>(bias);
    auto *R = static_cast<uint16_t *>(residual);
    auto *Y = static_cast<uint16_t *>(y);
    const unsigned gy = (unsigned)((M + kRows - 1) / kRows);
    const int m = (int)M, n = (int)N, k = (int)K, ld = (int)ldy;
    if (silu) {
        // W holds 2N rows (gate then up); each tile produces 8 outputs per 16-column block
        if (N % 8) return SWH_E_ARG;
        constexpr int NB = 16;
        const dim3 grid((unsigned)(N / (NB / 2)), gy);
        if (NW) decode_gemm_kernel<NB, true, EPI_SILU, false><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, nullptr, nullptr, Y, ld);
        else decode_gemm_kernel<NB, false, EPI_SILU, false><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, nullptr, nullptr, Y, ld);
        return launch_status();
    }
    if (residual) {
        constexpr int NB = 16;
        const dim3 grid((unsigned)((N + NB - 1) / NB), gy);
        if (N % 16) return SWH_E_ARG;
        if (NW) decode_gemm_kernel<NB, true, EPI_RESIDUAL, false><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, nullptr, R, nullptr, ld);
        else decode_gemm_kernel<NB, false, EPI_RESIDUAL, false><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, nullptr, R, nullptr, ld);
        return launch_status();
    }
    if (N % 16) return SWH_E_ARG;
    if (N >= 65536) {  // lm head: wide tiles keep the L2 re-reads of X below the W stream
        constexpr int NB = 64;
        if (N % NB) return SWH_E_ARG;
        const dim3 grid((unsigned)(N / NB), gy);
        if (NW) decode_gemm_kernel<NB, true, EPI_PLAIN, false><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, nullptr, nullptr, Y, ld);
        else decode_gemm_kernel<NB, false, EPI_PLAIN, false><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, nullptr, nullptr, Y, ld);
        return launch_status();
    }
    constexpr int NB = 16;
    const dim3 grid((unsigned)(N / NB), gy);
    if (NW && Bs) decode_gemm_kernel<NB, true, EPI_PLAIN, true><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, Bs, nullptr, Y, ld);
    else if (NW) decode_gemm_kernel<NB, true, EPI_PLAIN, false><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, nullptr, nullptr, Y, ld);
    else if (Bs) decode_gemm_kernel<NB, false, EPI_PLAIN, true><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, Bs, nullptr, Y, ld);
    else decode_gemm_kernel<NB, false, EPI_PLAIN, false><<<grid, kGemmThreads, 0, s>>>(X, W, m, n, k, NW, eps, nullptr, nullptr, Y, ld);
    return launch_status();
}
