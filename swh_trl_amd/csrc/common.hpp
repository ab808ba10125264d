// Shared device helpers for the swh_trl_amd HIP kernels (gfx950 / CDNA4).
// Wave width is 64 on CDNA; every reduction below is written for 64 lanes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/swh_trl_amd.h"

namespace swh {

constexpr int kWave = 64;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kNegInf = -__builtin_huge_valf();

// ---- bf16 <-> f32 -----------------------------------------------------------
__device__ __forceinline__ float bf16_bits_to_f32(uint32_t u16) { return __uint_as_float(u16 << 16); }

// Round-to-nearest-even, NaN stays NaN (clang lowers the __bf16 cast to
// v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ uint16_t f32_to_bf16_bits(float f) {
    __bf16 b = static_cast<__bf16>(f);
    return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float round_bf16(float f) { return bf16_bits_to_f32(f32_to_bf16_bits(f)); }

__device__ __forceinline__ float f16_bits_to_f32(uint32_t u16) {
    _Float16 h = __builtin_bit_cast(_Float16, (uint16_t)u16);
    return (float)h;
}
__device__ __forceinline__ uint16_t f32_to_f16_bits(float f) {
    _Float16 h = (_Float16)f;
    return __builtin_bit_cast(uint16_t, h);
}

template <int DT> struct Elem;
template <> struct Elem<SWH_F32> {
    using T = float;
    static __device__ __forceinline__ float load(const float *p) { return *p; }
    static __device__ __forceinline__ float round(float f) { return f; }
};
template <> struct Elem<SWH_BF16> {
    using T = uint16_t;
    static __device__ __forceinline__ float load(const uint16_t *p) { return bf16_bits_to_f32(*p); }
    static __device__ __forceinline__ float round(float f) { return round_bf16(f); }
};
template <> struct Elem<SWH_F16> {
    using T = uint16_t;
    static __device__ __forceinline__ float load(const uint16_t *p) { return f16_bits_to_f32(*p); }
    static __device__ __forceinline__ float round(float f) { return f16_bits_to_f32(f32_to_f16_bits(f)); }
};

// Unpack a 16-byte vector into floats: 8 x 16-bit or 4 x f32.
template <int DT> __device__ __forceinline__ void unpack16(const uint4 &v, float *out);
template <> __device__ __forceinline__ void unpack16<SWH_BF16>(const uint4 &v, float *o) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[2 * i] = __uint_as_float(w[i] << 16);
        o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
template <> __device__ __forceinline__ void unpack16<SWH_F16>(const uint4 &v, float *o) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[2 * i] = f16_bits_to_f32(w[i] & 0xffffu);
        o[2 * i + 1] = f16_bits_to_f32(w[i] >> 16);
    }
}
template <> __device__ __forceinline__ void unpack16<SWH_F32>(const uint4 &v, float *o) {
    o[0] = __uint_as_float(v.x);
    o[1] = __uint_as_float(v.y);
    o[2] = __uint_as_float(v.z);
    o[3] = __uint_as_float(v.w);
}
template <int DT> constexpr int kPerVec = (DT == SWH_F32) ? 4 : 8;

// ---- 16-byte streaming loads/stores (non-temporal: read-once rows) ---------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4 *p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return uint4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void st_nt(uint4 *p, const uint4 &v) {
    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4 *>(p));
}

// Visit elements [begin, end) of a row with `nthreads` cooperating threads,
// 16-byte vector loads in the aligned body: f(j, x) with x the f32 value.
template <int DT, bool NT, typename F>
__device__ __forceinline__ void row_foreach(const typename Elem<DT>::T *row, int64_t begin, int64_t end, int tid,
                                            int nthreads, F &&f) {
    using T = typename Elem<DT>::T;
    constexpr int PV = kPerVec<DT>;
    if (end <= begin) return;
    const uintptr_t a = reinterpret_cast<uintptr_t>(row + begin);
    int64_t head = (int64_t)(((16 - (a & 15)) & 15) / sizeof(T));
    if ((a & (sizeof(T) - 1)) != 0) head = end - begin;  // not even element-aligned: scalar
    if (head > end - begin) head = end - begin;
    for (int64_t j = begin + tid; j < begin + head; j += nthreads) f(j, Elem<DT>::load(row + j));
    const int64_t b0 = begin + head;
    const int64_t nvec = (end - b0) / PV;
    const uint4 *vp = reinterpret_cast<const uint4 *>(row + b0);
    // four grid-strided vectors per trip, all loads issued before any use: a
    // workgroup walking a long row alone keeps 4 loads in flight per thread
    constexpr int U = 4;
    int64_t v = tid;
    for (; v + (U - 1) * (int64_t)nthreads < nvec; v += U * (int64_t)nthreads) {
        uint4 raw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (NT) raw[u] = ld_nt(vp + v + u * nthreads);
            else raw[u] = vp[v + u * nthreads];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float x[PV];
            unpack16<DT>(raw[u], x);
            const int64_t j0 = b0 + (v + u * nthreads) * PV;
#pragma unroll
            for (int k = 0; k < PV; ++k) f(j0 + k, x[k]);
        }
    }
    for (; v < nvec; v += nthreads) {
        float x[PV];
        uint4 raw;
        if constexpr (NT) raw = ld_nt(vp + v);
        else raw = vp[v];
        unpack16<DT>(raw, x);
        const int64_t j0 = b0 + v * PV;
#pragma unroll
        for (int k = 0; k < PV; ++k) f(j0 + k, x[k]);
    }
    for (int64_t j = b0 + nvec * PV + tid; j < end; j += nthreads) f(j, Elem<DT>::load(row + j));
}

// ---- fast transcendental helpers (v_exp_f32 / v_log_f32 are base-2) --------
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * kLog2e); }
__device__ __forceinline__ float fast_log(float x) { return __builtin_amdgcn_logf(x) * kLn2; }

// ---- wave / block reductions ------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// Block-wide sum of NV floats; result broadcast to every thread.  `red` must
// hold NV * (blockDim.x / 64) floats.  Deterministic order.
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float *red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) red[k * nw + wid] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float s = 0.f;
        for (int w = 0; w < nw; ++w) s += red[k * nw + w];
        v[k] = s;
    }
    __syncthreads();
}

template <int NV>
__device__ __forceinline__ void block_sum_d(double (&v)[NV], double *red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_sum_d(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) red[k * nw + wid] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = 0.0;
        for (int w = 0; w < nw; ++w) s += red[k * nw + w];
        v[k] = s;
    }
    __syncthreads();
}

// ---- online softmax state: (max, sum e^{z-m}, sum e^{z-m}(z-m)) -------------
struct SoftState {
    float m, s1, s2;
};
__device__ __forceinline__ SoftState soft_init() { return {kNegInf, 0.f, 0.f}; }

// Branch-free online (max, sum e^(z - max)) fold of one value for the streaming
// draw passes (no entropy term; z may be -inf).  Equal to soft_fold<1>'s (m, s1):
// for z <= m the rescale factor is e^0 = 1; the clamps turn the -inf - -inf NaNs of
// an empty state into e^-1e4 = 0.  Multiply and add stay separate roundings, as there.
__device__ __forceinline__ void soft_fold1(float &m, float &s1, float z) {
    const float mn = fmaxf(m, z);
    const float f = fast_exp(fmaxf(m - mn, -1.0e4f)), e = fast_exp(fmaxf(z - mn, -1.0e4f));
    s1 = __fadd_rn(__fmul_rn(s1, f), e);
    m = mn;
}

// Merge b into a.
__device__ __forceinline__ SoftState soft_merge(SoftState a, SoftState b) {
    if (b.m == kNegInf) return a;
    if (a.m == kNegInf) return b;
    const float M = fmaxf(a.m, b.m);
    const float da = a.m - M, db = b.m - M;
    const float fa = fast_exp(da), fb = fast_exp(db);
    SoftState r;
    r.m = M;
    r.s1 = fa * a.s1 + fb * b.s1;
    r.s2 = fa * (a.s2 + da * a.s1) + fb * (b.s2 + db * b.s1);
    return r;
}

// Fold N values (already processed) into the state.
template <int N>
__device__ __forceinline__ void soft_fold(SoftState &st, const float *z) {
    float lm = z[0];
#pragma unroll
    for (int k = 1; k < N; ++k) lm = fmaxf(lm, z[k]);
    if (lm == kNegInf) return;
    if (lm > st.m) {
        if (st.m == kNegInf) {
            st.s1 = 0.f;
            st.s2 = 0.f;
        } else {
            const float d = st.m - lm;
            const float f = fast_exp(d);
            st.s2 = f * (st.s2 + d * st.s1);
            st.s1 = f * st.s1;
        }
        st.m = lm;
    }
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const float d = fmaxf(z[k] - st.m, -1.0e4f);
        const float e = fast_exp(d);
        st.s1 += e;
        st.s2 = fmaf(e, d, st.s2);
    }
}

__device__ __forceinline__ SoftState wave_soft(SoftState s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        SoftState t;
        t.m = __shfl_xor(s.m, o, kWave);
        t.s1 = __shfl_xor(s.s1, o, kWave);
        t.s2 = __shfl_xor(s.s2, o, kWave);
        s = soft_merge(s, t);
    }
    return s;
}

// Block-wide merge; `red` holds 3 * nwaves floats.  Result broadcast.
__device__ __forceinline__ SoftState block_soft(SoftState s, float *red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    s = wave_soft(s);
    if (lane == 0) {
        red[wid] = s.m;
        red[nw + wid] = s.s1;
        red[2 * nw + wid] = s.s2;
    }
    __syncthreads();
    SoftState r = soft_init();
    for (int w = 0; w < nw; ++w) r = soft_merge(r, SoftState{red[w], red[nw + w], red[2 * nw + w]});
    __syncthreads();
    return r;
}

// ---- Philox4x32-10 (Salmon et al. SC'11); matches oracle/c/philox_ref.c ----
// one (row, workgroup) partial of the fused lm-head samplers: the best Gumbel key and its column
struct LmPart {
    float key;
    int32_t idx;
};

struct U4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        // one v_mad_u64_u32 per product (both halves) instead of v_mul_lo_u32 + v_mul_hi_u32
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    }
    return c;
}
__device__ __forceinline__ float u01_from_bits(uint32_t w) {
    return ((float)(w >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// Gumbel noise g = -log(-log u) of the uniform u = ((w >> 8) + 0.5) 2^-24 (the sampler
// stream, oracle/c/philox_ref.c).  For u within a few 2^-24 of 1, v_log_f32(u) returns 0
// and -log(0) made g = +inf: that element won the draw whatever its logit (about 1 % of
// the rows of a 151936-wide step).  There -log(u) = -log(1 - d) is taken from its series
// in d = 1 - u (exact in fp32: ((2^24 - 1 - (w >> 8)) + 0.5) 2^-24), d + d^2/2 + d^3/3,
// whose next term is below 2^-23 relative for d < 2^-7.
__device__ __forceinline__ float gumbel_from_bits(uint32_t w) {
    const uint32_t m = w >> 8;
    const float u = ((float)m + 0.5f) * (1.0f / 16777216.0f);
    const float d = ((float)(16777215u - m) + 0.5f) * (1.0f / 16777216.0f);
    // both branches evaluated, one select: a divergent branch here cost the streaming draw
    // passes more than the series
    const float ts = d * fmaf(d, fmaf(d, 1.0f / 3.0f, 0.5f), 1.0f), tl = -fast_log(u);
    return -fast_log(d < 0.0078125f ? ts : tl);
}

// ---- launch helpers -----------------------------------------------------------
inline int launch_status() { return hipGetLastError() == hipSuccess ? SWH_OK : SWH_E_LAUNCH; }

// ---- the library's host-side state (csrc/lib.hip) ------------------------------
// Per-device facts, each queried once per device under std::call_once, and the
// calling thread's launch policy of swh_set_launch_policy (thread_local).  Nothing
// else in the library outlives a call, and nothing reads the environment.
constexpr int kMaxDevices = 64;
constexpr int kMaxDynLds = 160 * 1024;  // gfx950 LDS per workgroup

int cu_count();                        // current device's CUs (256 if the query fails)
swh_launch_policy launch_policy();     // the calling thread's policy
bool lds_opt_in_once(const void *kernel, std::once_flag *once, bool *ok);

// Opt a kernel into > 64 KB of dynamic LDS, once per (kernel, device): the
// attribute is per device, so the flags are a per-device table per kernel.
template <auto Kernel>
bool lds_opt_in() {
    static std::once_flag once[kMaxDevices];
    static bool ok[kMaxDevices];
    return lds_opt_in_once(reinterpret_cast<const void *>(Kernel), once, ok);
}

}  // namespace swh
