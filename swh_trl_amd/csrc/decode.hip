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
// grid = (column blocks, M tiles, S k-splits).  The 4*S waves of a column
// block split its K/32 k-steps evenly.  S > 1: every workgroup publishes its
// [64 x NB] fp32 partial with write-through (sc1) stores, drains, and one lane
// takes a ticket on the block's counter (agent-scope atomic); the workgroup
// that draws S-1 sums the S slabs in fixed order (sc1 loads: deterministic,
// placement-independent — MI355X_MICROARCH.md §Workgroup dispatch, table row 1)
// and runs the epilogue, then resets the counter for the next launch.
constexpr int kU = 4;  // k-steps whose loads are issued together
constexpr int kMaxNormK = 8192;
constexpr int64_t kCounterBytes = 1 << 16;  // split-K ticket counters (16384 column blocks)

template <int NB, bool NORM, int EPI, bool BIAS>
__global__ __launch_bounds__(kGemmThreads) void decode_gemm_kernel(
    const uint16_t *__restrict__ x, const uint16_t *__restrict__ w, int M, int N, int K,
    const uint16_t *__restrict__ norm_w, float eps, const uint16_t *__restrict__ bias, uint16_t *__restrict__ res,
    uint16_t *__restrict__ y, int ldy, float *__restrict__ slabs, int *__restrict__ counters) {
    constexpr int CB = NB / 16;
    __shared__ float rstd_s[kRows];
    __shared__ float part[4][kRows][NB + 1];
    __shared__ uint4 nw_s[NORM ? kMaxNormK / 8 : 1];  // RMSNorm weight, staged once
    __shared__ int last_s;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int S = gridDim.z, sidx = blockIdx.z;
    const int m0 = blockIdx.y * kRows;
    const int n0 = blockIdx.x * (EPI == EPI_SILU ? NB / 2 : NB);

    // ---- prologue: per-row rstd of X, 4 threads per row, loads issued in bulk
    if constexpr (NORM) {
        const int r = tid >> 2, q = tid & 3;
        const int gr = min(m0 + r, M - 1);
        const int nv = K / 8, v0 = q * (nv / 4), v1 = (q == 3) ? nv : v0 + nv / 4;
        const uint4 *xr = reinterpret_cast<const uint4 *>(x + (int64_t)gr * K);
        float ss = 0.f;
        int v = v0;
        for (; v + 8 <= v1; v += 8) {
            uint4 t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] = xr[v + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                float a[8];
                unpack16<SWH_BF16>(t[u], a);
#pragma unroll
                for (int k = 0; k < 8; ++k) ss = fmaf(a[k], a[k], ss);
            }
        }
        for (; v < v1; ++v) {
            float a[8];
            unpack16<SWH_BF16>(xr[v], a);
#pragma unroll
            for (int k = 0; k < 8; ++k) ss = fmaf(a[k], a[k], ss);
        }
        ss += __shfl_xor(ss, 1, kWave);
        ss += __shfl_xor(ss, 2, kWave);
        if (q == 0) rstd_s[r] = rsqrtf(ss / (float)K + eps);
        for (int i = tid; i < K / 8; i += kGemmThreads) nw_s[i] = reinterpret_cast<const uint4 *>(norm_w)[i];
        __syncthreads();
    }

    // ---- main loop over this wave's k-steps
    const int KS = K / 32, parts = 4 * S, pidx = sidx * 4 + wid;
    const int ks0 = (int)((int64_t)KS * pidx / parts), ks1 = (int)((int64_t)KS * (pidx + 1) / parts);
    const int rl = lane & 15, kq = (lane >> 4) * 8;
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
        xrow[i] = x + (int64_t)r * K + kq;
        rs[i] = NORM ? rstd_s[i * 16 + rl] : 1.f;
    }
    const uint16_t *wrow[CB];
#pragma unroll
    for (int j = 0; j < CB; ++j) {
        int n;
        if constexpr (EPI == EPI_SILU) {
            const int c = j * 8 + (rl & 7);
            n = (rl < 8) ? n0 + c : N + n0 + c;
        } else {
            n = n0 + j * 16 + rl;
        }
        wrow[j] = w + (int64_t)n * K + kq;
    }
    auto mma_step = [&](const uint4 (&av)[4], const uint4 (&bv)[CB], int kk) {
        uint4 a2[4];
        if constexpr (NORM) {
            const uint4 nw = nw_s[(kk + kq) >> 3];
#pragma unroll
            for (int i = 0; i < 4; ++i) a2[i] = norm_frag(av[i], nw, rs[i]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) a2[i] = av[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < CB; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a2[i]), as_bf16x8(bv[j]), acc[i][j], 0,
                                                                    0, 0);
    };
    int ks = ks0;
    for (; ks + kU <= ks1; ks += kU) {
        uint4 bv[kU][CB], av[kU][4];
#pragma unroll
        for (int u = 0; u < kU; ++u)
#pragma unroll
            for (int j = 0; j < CB; ++j) bv[u][j] = ld_nt(reinterpret_cast<const uint4 *>(wrow[j] + (ks + u) * 32));
#pragma unroll
        for (int u = 0; u < kU; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) av[u][i] = *reinterpret_cast<const uint4 *>(xrow[i] + (ks + u) * 32);
#pragma unroll
        for (int u = 0; u < kU; ++u) mma_step(av[u], bv[u], (ks + u) * 32);
    }
    for (; ks < ks1; ++ks) {
        uint4 bv[CB], av[4];
#pragma unroll
        for (int j = 0; j < CB; ++j) bv[j] = ld_nt(reinterpret_cast<const uint4 *>(wrow[j] + ks * 32));
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = *reinterpret_cast<const uint4 *>(xrow[i] + ks * 32);
        mma_step(av, bv, ks * 32);
    }

    // ---- merge the 4 waves in LDS -> part[0]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) part[wid][i * 16 + (lane >> 4) * 4 + e][j * 16 + rl] = acc[i][j][e];
    __syncthreads();
    for (int idx = tid; idx < kRows * NB; idx += kGemmThreads) {
        const int r = idx / NB, c = idx - r * NB;
        part[0][r][c] = part[0][r][c] + part[1][r][c] + part[2][r][c] + part[3][r][c];
    }
    __syncthreads();

    // ---- cross-workgroup split-K: publish, ticket, last arriver reduces
    if (S > 1) {
        const int blk = blockIdx.y * gridDim.x + blockIdx.x;
        float *my = slabs + ((int64_t)blk * S + sidx) * (kRows * NB);
        for (int idx = tid; idx < kRows * NB; idx += kGemmThreads)
            __hip_atomic_store(my + idx, part[0][idx / NB][idx % NB], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const int t = __hip_atomic_fetch_add(counters + blk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last_s = (t == S - 1);
        }
        __syncthreads();
        if (!last_s) return;
        const float *base = slabs + (int64_t)blk * S * (kRows * NB);
        for (int idx = tid; idx < kRows * NB; idx += kGemmThreads) {
            float v = 0.f;
            for (int q = 0; q < S; ++q)
                v += __hip_atomic_load(base + (int64_t)q * kRows * NB + idx, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            part[0][idx / NB][idx % NB] = v;
        }
        if (tid == 0) __hip_atomic_store(counters + blk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
    }

    // ---- epilogue
    if constexpr (EPI == EPI_SILU) {
        constexpr int NO = NB / 2;
        for (int idx = tid; idx < kRows * NO; idx += kGemmThreads) {
            const int r = idx / NO, c = idx - r * NO;
            const int gr = m0 + r;
            if (gr >= M) continue;
            const int jb = c / 8, cc = c - jb * 8;
            const int cg = jb * 16 + cc;
            const float g = round_bf16(part[0][r][cg]), u = round_bf16(part[0][r][cg + 8]);
            const float a = round_bf16(g / (1.f + expf(-g))) * u;
            y[(int64_t)gr * ldy + n0 + c] = f32_to_bf16_bits(a);
        }
    } else {
        for (int idx = tid; idx < kRows * NB; idx += kGemmThreads) {
            const int r = idx / NB, c = idx - r * NB;
            const int gr = m0 + r, gc = n0 + c;
            if (gr >= M || gc >= N) continue;
            float v = part[0][r][c];
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

extern "C" int64_t swh_decode_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
    const int64_t mt = (M + kRows - 1) / kRows;
    const int64_t ncb = (N + 15) / 16;
    const int64_t S = 16;  // upper bound of the split the host picks
    return kCounterBytes + mt * ncb * S * kRows * 16 * (int64_t)sizeof(float);
    (void)K;
}

namespace swh {
namespace {
// split-K factor: aim at >= ~384 workgroups with >= 2 k-steps per wave
int pick_split(int64_t blocks, int64_t K) {
    const int64_t KS = K / 32;
    int64_t S = (384 + blocks - 1) / blocks;
    if (S > KS / 8) S = KS / 8;
    if (S > 16) S = 16;
    return S < 1 ? 1 : (int)S;
}
}  // namespace
}  // namespace swh

extern "C" int swh_decode_gemm(const void *x, const void *w, int64_t M, int64_t N, int64_t K, const void *norm_w,
                               float eps, const void *bias, void *residual, int32_t silu, void *y, int64_t ldy,
                               void *workspace, int64_t workspace_bytes, void *stream) {
    if (!x || !w || M <= 0 || N <= 0 || K <= 0 || K % 32 || M > (1 << 20) || N >= (1 << 30) || K >= (1 << 30))
        return SWH_E_ARG;
    if (residual && (silu || bias)) return SWH_E_ARG;
    if (!residual && !y) return SWH_E_ARG;
    if (((uintptr_t)x | (uintptr_t)w) & 15) return SWH_E_ARG;
    if (norm_w && (((uintptr_t)norm_w & 15) || K > kMaxNormK)) return SWH_E_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const auto *X = static_cast<const uint16_t *>(x);
    const auto *W = static_cast<const uint16_t *>(w);
    const auto *NW = static_cast<const uint16_t *>(norm_w);
    const auto *Bs = static_cast<const uint16_t *>(bias);
    auto *R = static_cast<uint16_t *>(residual);
    auto *Y = static_cast<uint16_t *>(y);
    const unsigned gy = (unsigned)((M + kRows - 1) / kRows);
    const int m = (int)M, n = (int)N, k = (int)K, ld = (int)ldy;
    // workspace: [counters (zeroed, int32) | slabs (fp32)]
    int *ctr = static_cast<int *>(workspace);
    float *slab = nullptr;
    auto prep = [&](int64_t blocks, int S, int nb) -> bool {
        if (S == 1) return true;
        const int64_t need = kCounterBytes + blocks * gy * S * kRows * nb * 4;
        if (blocks * gy * (int64_t)sizeof(int) > kCounterBytes) return false;
        if (!workspace || workspace_bytes < need) return false;
        // counters live in a FIXED region at the start (never overlapped by any
        // call's slabs, whatever its shape), so a self-reset counter stays zero
        slab = reinterpret_cast<float *>(static_cast<char *>(workspace) + kCounterBytes);
        return true;
    };
#define SWH_GEMM(NB_, NORM_, EPI_, BIAS_, GX, S_)                                                                  \
    decode_gemm_kernel<NB_, NORM_, EPI_, BIAS_><<<dim3((unsigned)(GX), gy, (unsigned)(S_)), kGemmThreads, 0, s>>>( \
        X, W, m, n, k, NW, eps, Bs, R, Y, ld, slab, ctr)
    if (silu) {
        if (N % 8) return SWH_E_ARG;
        const int64_t blocks = N / 8;
        const int S = pick_split(blocks, K);
        if (!prep(blocks, S, 16)) return SWH_E_ARG;
        if (NW) SWH_GEMM(16, true, EPI_SILU, false, blocks, S);
        else SWH_GEMM(16, false, EPI_SILU, false, blocks, S);
        return launch_status();
    }
    if (N % 16) return SWH_E_ARG;
    if (residual) {
        const int64_t blocks = N / 16;
        const int S = pick_split(blocks, K);
        if (!prep(blocks, S, 16)) return SWH_E_ARG;
        if (NW) SWH_GEMM(16, true, EPI_RESIDUAL, false, blocks, S);
        else SWH_GEMM(16, false, EPI_RESIDUAL, false, blocks, S);
        return launch_status();
    }
    if (N >= 65536 && N % 64 == 0) {  // lm head: wide tiles keep X re-reads below the W stream
        const int64_t blocks = N / 64;
        if (NW) SWH_GEMM(64, true, EPI_PLAIN, false, blocks, 1);
        else SWH_GEMM(64, false, EPI_PLAIN, false, blocks, 1);
        return launch_status();
    }
    const int64_t blocks = N / 16;
    const int S = pick_split(blocks, K);
    if (!prep(blocks, S, 16)) return SWH_E_ARG;
    if (NW && Bs) SWH_GEMM(16, true, EPI_PLAIN, true, blocks, S);
    else if (NW) SWH_GEMM(16, true, EPI_PLAIN, false, blocks, S);
    else if (Bs) SWH_GEMM(16, false, EPI_PLAIN, true, blocks, S);
    else SWH_GEMM(16, false, EPI_PLAIN, false, blocks, S);
#undef SWH_GEMM
    return launch_status();
}
