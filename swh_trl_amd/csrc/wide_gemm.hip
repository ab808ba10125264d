// Streamed decode GEMM for the bandwidth regime (Llama-3-8B decode at 64 rows,
// BASELINE.json config 5): Y[M <= 64, N] = X[M, K] W[N, K]^T with K >= 2048.
//
// Why a second decode GEMM: decode_gemm stages a workgroup's whole X slice
// [rows x K/S] in LDS, so at 64 rows and K = 4096 / 14336 it must tile the
// rows by 16 (every weight byte then crosses the CU load path once per row
// tile) or split K many ways; at 8B that ran the decode projections at
// 1.6-2 TB/s.  Here a workgroup owns 128 weight rows (32 per wave) for ALL 64
// rows over a K range, and both operands stream through a 3-slot LDS ring in
// 128-k rounds by LDS-DMA (two rounds in flight while one is computed;
// XOR-swizzled 16-B pieces so the 16 rows an MFMA fragment reads sit in
// distinct banks): every weight byte is read from HBM once, X (L2-resident)
// once per workgroup.  v_mfma_f32_16x16x32_bf16, A = X rows, B = weight rows.
// K is split over S workgroups only as far as needed to fill the CUs; the S
// fp32 tiles meet through write-through slabs and an agent-scope ticket (the
// last arriver sums them in fixed order: deterministic), no spin-waits.
// Epilogues as decode_gemm: plain (+ bias) with the folded-RMSNorm row scale
// rstd from the producer's partial sums (ss_in), residual (+ the next norm's
// partial sums ss_out), SiLU gate.
#include <cstdlib>

#include "common.hpp"

namespace swh {

int wide_gemm(const void *x, const void *w, int64_t M, int64_t N, int64_t K, float eps, const float *ss_in,
              const void *bias, void *residual, int32_t silu, void *y, int64_t ldy, float *ss_out, void *workspace,
              int64_t workspace_bytes, int64_t counter_bytes, int32_t packed, hipStream_t stream);
int64_t wide_gemm_slab_bytes(int64_t M, int64_t N, int64_t K, int32_t silu);
bool wide_gemm_eligible(int64_t M, int64_t N, int64_t K, int32_t silu);
int wide_pack(const void *src, const void *norm_w, int64_t N, int64_t K, int32_t silu, void *dst, hipStream_t stream);
int wide_lm_sample(const void *x, const void *w, int64_t M, int64_t V, int64_t K, float eps, const float *ss_in,
                   const swh_sample_params &p, const uint64_t *rng, const int32_t *step, LmPart *part, int *pstride,
                   hipStream_t stream);

namespace {

typedef __bf16 bf16x8w __attribute__((ext_vector_type(8)));
typedef float f32x4w __attribute__((ext_vector_type(4)));

constexpr int kWW = 8;                 // waves per workgroup (the widest geometry)
constexpr int kWKS = 4;                // k-steps (of 32) per round
constexpr int kWKC = 32 * kWKS;        // k per round: 128 (256-B rows of 16 pieces)
constexpr int kWXB = 64 * kWKC * 2;    // X bytes of a round (16 KB)
constexpr int kWXP = kWXB / 16;        // X pieces of a round (1024)

// Geometry per CB = 16-row weight groups per wave and W = waves: a workgroup owns
// NB = 16 CB W weight rows.  CB 2 halves the X bytes every workgroup ingests per weight
// byte (the wide-N shapes: Llama-3-8B lm head); its ring is 4 rounds deep (VGPR budget:
// 40 registers per round against 24).  W 7 / 6 make tile counts that fill the CUs where
// 8 waves leave some idle (gate/up: 224 tiles of 128 rows, 256 of 112; qkv: 48 x 5
// splits, 64 x 4 of 96 rows).
template <int CB, int W = kWW>
struct WGeo {
    static constexpr int T = 64 * W;                     // threads
    static constexpr int NB = 16 * CB * W;
    static constexpr int XU = (kWXP + T - 1) / T;        // X pieces per thread per round (2 or 3)
    static constexpr int D = CB == 1 ? (XU == 2 ? 7 : 6) : 4;  // rounds in flight (register ring depth)
    static constexpr int LDT = NB + 4;                   // epilogue tile row stride (f32)
    // the epilogue tile, which the two X slots live under, then rstd + flag
    static constexpr int AUX = 64 * LDT * 4 > 2 * kWXB ? 64 * LDT * 4 : 2 * kWXB;
    static constexpr int LDS = AUX + 64 * 4 + 16;
};
constexpr int kWNB = 16 * kWW;  // the 8-wave tile: eligibility (wcols % 128)

enum : int { WEPI_PLAIN = 0, WEPI_RESIDUAL = 1, WEPI_SILU = 2, WEPI_SAMPLE = 3, WEPI_SAMPLE_T = 4 };

// The fused lm-head sampler's operands (WEPI_SAMPLE: the unfiltered swh_sample_step per
// element of the tile, _T with the temperature division): one LmPart per (row, workgroup).
struct WSample {
    swh_sample_params p;
    const uint64_t *rng;
    const int32_t *step;
    LmPart *part;  // [M][pstride]
    int pstride;
};

// Phase timestamps for tools/wide_probe.py (a build with SWH_WIDE_TRACE_ON defined,
// tools/build_variant.py): wall clock (100 MHz) of thread 0 at each phase boundary.
#ifdef SWH_WIDE_TRACE_ON
__device__ unsigned long long *g_wide_trace;
#define SWH_WIDE_TRACE(i)                                                                                      \
    if (threadIdx.x == 0 && g_wide_trace)                                                                      \
    g_wide_trace[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = wall_clock64()
#else
#define SWH_WIDE_TRACE(i)
#endif

__device__ __forceinline__ bf16x8w as_bf8(const uint4 &v) { return __builtin_bit_cast(bf16x8w, v); }

// Weight fragments are read once per launch: non-temporal loads keep the weight stream from
// evicting X (re-read by every workgroup of an XCD) and the slabs from L2 (Llama-3-8B decode,
// tools/wide_probe.py: gate/up 52 -> 48.4 us, down 29.1 -> 27.4, lm head 199 -> 184).
__device__ __forceinline__ uint4 wload_nt(const uint16_t *p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return uint4{v.x, v.y, v.z, v.w};
}

// barrier that waits for LDS traffic only: LDS-DMA still in flight stays in flight
__device__ __forceinline__ void wide_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ uint4 pack8w(const float *v) {
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        o[k] = (uint32_t)f32_to_bf16_bits(v[2 * k]) | ((uint32_t)f32_to_bf16_bits(v[2 * k + 1]) << 16);
    return uint4{o[0], o[1], o[2], o[3]};
}

// NM: 0 = plain X, 2 = folded RMSNorm (rstd row scale from ss_in in the epilogue).
// PACKED: the weight is in the fragment order wide_pack writes (below): a wave's
// 16 rows x 128 k of a round are one contiguous 4 KB run and each load
// instruction of the wave reads 1 KB of it, instead of 16 rows x 64 B 8 KB
// (K x 2 B) apart; same k-slot mapping, so the results are bit-identical.
// Plain register loads only (no LDS-DMA: hipcc drains vmcnt(0) at the use of
// any register load while an LDS-DMA is in flight — cdna_hip_programming.md,
// LDS-DMA notes), so the compiler's counted waits keep WD - 1 rounds in
// flight; one LDS array (a second __shared__ object makes hipcc wait before
// LDS reads).
template <int EPI, int NM, bool BIAS, bool PACKED, int CB, int W>
__global__ __launch_bounds__(64 * W) void wide_gemm_kernel(const uint16_t *__restrict__ x, const uint16_t *__restrict__ w,
                                                        int M, int N, int K, float eps, const float *__restrict__ ss_in,
                                                        const uint16_t *__restrict__ bias, uint16_t *__restrict__ res,
                                                        float *__restrict__ ss_out, uint16_t *__restrict__ y, int ldy,
                                                        float *__restrict__ slabs, int *__restrict__ counters,
                                                        WSample smp) {
    using G = WGeo<CB, W>;
    constexpr int NB = G::NB, WD = G::D, LDT = G::LDT, AUX = G::AUX, kWT = G::T, kWXU = G::XU;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float *rstd_s = reinterpret_cast<float *>(lds + AUX);
    int *flag_s = reinterpret_cast<int *>(lds + AUX + 64 * 4);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, rl = lane & 15, kg = lane >> 4;
    const int S = gridDim.y, sidx = blockIdx.y, cb = blockIdx.x;
    const int nr_all = K / kWKC;
    const int r0 = (int)((int64_t)nr_all * sidx / S), r1 = (int)((int64_t)nr_all * (sidx + 1) / S), nr = r1 - r0;
    const int kbase = r0 * kWKC;
    SWH_WIDE_TRACE(0);

    // ---- the folded norm's row statistic (L2)
    if constexpr (NM == 2) {
        // 8 lanes per row, 16-B loads 8 deep: one memory latency (a scalar walk of the
        // row's K / 16 partial sums took 5-6 us at K 4096)
        const int sub = tid & 7, nc4 = K / 64;
        for (int r = tid >> 3; r < 64; r += kWT / 8) {  // whole 8-lane groups per row
            const float4 *row = reinterpret_cast<const float4 *>(ss_in + (int64_t)min(r, M - 1) * (K / 16));
            float4 a = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
            for (int f = sub; f < nc4; f += 8) {
                const float4 t = row[f];
                a.x += t.x;
                a.y += t.y;
                a.z += t.z;
                a.w += t.w;
            }
            float v = (a.x + a.y) + (a.z + a.w);
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            if (sub == 0) rstd_s[r] = rsqrtf(v / (float)K + eps);
        }
    }

    // ---- operands: a register ring WD rounds deep per thread (X pieces + this wave's weight
    // fragments; plain loads, so hipcc counts vmcnt per round), X then copied into one of two
    // LDS slots per round.  LDS piece (row, p) holds X piece (row, p ^ (row & 15)): the 16 rows
    // an MFMA fragment reads sit in distinct banks.  Tile row t -> weight row: wave t / 16,
    // lane t % 16; SiLU tiles pair gate rows (lanes 0-7) with the matching up rows (lanes 8-15).
    auto wrow_of = [&](int t) -> int {
        if constexpr (EPI == WEPI_SILU) {
            const int oc = cb * (NB / 2) + (t >> 4) * 8 + (t & 7);
            return (t & 15) < 8 ? oc : N + oc;
        } else {
            return cb * NB + t;
        }
    };
    // weight element strides of a round and of a k-step in the two layouts
    constexpr int kRS = PACKED ? 16 * kWKC : kWKC, kSS = PACKED ? 16 * 32 : 32;
    const uint16_t *wp[CB];
#pragma unroll
    for (int j = 0; j < CB; ++j) {
        if constexpr (PACKED) {
            const int64_t bw = (int64_t)cb * (NB / 16) + wid * CB + j;  // 16-row group in tile order
            wp[j] = w + (bw * nr_all + r0) * (16 * kWKC) + (kg * 16 + rl) * 8;
        } else {
            wp[j] = w + (int64_t)wrow_of(wid * 16 * CB + 16 * j + rl) * K + kbase + 8 * kg;
        }
    }
    const uint16_t *xp[kWXU];
#pragma unroll
    for (int u = 0; u < kWXU; ++u) {  // pieces past the round (W 6 / 7) repeat the last one, never stored
        const int id = min(tid + kWT * u, kWXP - 1), row = id >> 4;
        xp[u] = x + (int64_t)min(row, M - 1) * K + kbase + (id & 15) * 8;
    }
    u32x4 xr[WD][kWXU];  // vector type, not the uint4 struct: an aggregate copy kept the ring in scratch
    uint4 wr[WD][kWKS][CB];
#define SWH_WIDE_ISSUE(q, D)                                                                                    \
    do {                                                                                                        \
        _Pragma("unroll") for (int u = 0; u < kWXU; ++u) xr[D][u] =                                            \
            *reinterpret_cast<const u32x4 *>(xp[u] + (q) * kWKC);                                               \
        _Pragma("unroll") for (int s = 0; s < kWKS; ++s) _Pragma("unroll") for (int j = 0; j < CB; ++j)       \
            wr[D][s][j] = wload_nt(wp[j] + (q) * kRS + kSS * s);                                                 \
        __builtin_amdgcn_sched_barrier(0); /* rounds issue in order: the counted waits rely on it */            \
    } while (0)
    f32x4w acc[4][CB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j) acc[i][j] = f32x4w{0.f, 0.f, 0.f, 0.f};
    // one round: X(r) into LDS slot r & 1, barrier, 4 k-steps x 4 row blocks of MFMAs, refill
    // the registers round r used with round r + WD
#define SWH_WIDE_ROUND(r, D, REFILL)                                                                            \
    do {                                                                                                        \
        unsigned char *xs = lds + ((r) & 1) * kWXB;                                                             \
        _Pragma("unroll") for (int u = 0; u < kWXU; ++u) {                                                      \
            const int id = tid + kWT * u, row = id >> 4;                                                        \
            if (kWXU * kWT == kWXP || id < kWXP)                                                                \
                *reinterpret_cast<u32x4 *>(xs + row * (kWKC * 2) + (((id & 15) ^ (row & 15)) * 16)) = xr[D][u]; \
        }                                                                                                       \
        wide_lds_barrier(); /* X(r) visible; every wave has left round r - 2 (same slot) */                     \
        _Pragma("unroll") for (int s = 0; s < kWKS; ++s) {                                                      \
            uint4 a[4];                                                                                         \
            _Pragma("unroll") for (int i = 0; i < 4; ++i) a[i] =                                                \
                *reinterpret_cast<const uint4 *>(xs + (16 * i + rl) * (kWKC * 2) + (((4 * s + kg) ^ rl) * 16));  \
            _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < CB; ++j)      \
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(a[i]), as_bf8(wr[D][s][j]),          \
                                                                    acc[i][j], 0, 0, 0);                         \
        }                                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                                      \
        if (REFILL) SWH_WIDE_ISSUE((r) + WD, D);                                                               \
    } while (0)
    int rb = 0;
    if (nr % WD == 0) {
        // a whole number of WD-round blocks: the prologue, the steady loop and the last WD
        // rounds are one fixed, branch-free pattern, and hipcc's counted waits keep WD - 1
        // rounds in flight to the end (lm head, down: 2-3 % faster than the tail below)
#pragma unroll
        for (int d = 0; d < WD; ++d) SWH_WIDE_ISSUE(d, d);
        for (; rb + WD < nr; rb += WD) {
#pragma unroll
            for (int d = 0; d < WD; ++d) SWH_WIDE_ROUND(rb + d, d, true);
        }
#pragma unroll
        for (int d = 0; d < WD; ++d) SWH_WIDE_ROUND(rb + d, d, false);
    } else {
        // The `if (r < nr)` tail makes the wait analysis merge paths: it waits for every load
        // each tail round (one round in flight).  Padding nr up to a multiple of WD with
        // masked rounds removes that but costs more than it saves when the padding is large
        // (o at 4 rounds: 16.0 -> 18.0 us; gate/up 32 -> 35 rounds: 58.2 -> 59.1 us).
        if (nr >= 2 * WD) {
            // unconditional prologue and steady state: every refill is in range, so the counted
            // waits see one fixed pattern at the loop header (WD - 1 rounds stay in flight)
#pragma unroll
            for (int d = 0; d < WD; ++d) SWH_WIDE_ISSUE(d, d);
            for (; rb + 2 * WD <= nr; rb += WD) {
#pragma unroll
                for (int d = 0; d < WD; ++d) SWH_WIDE_ROUND(rb + d, d, true);
            }
        } else {
#pragma unroll
            for (int d = 0; d < WD; ++d)
                if (d < nr) SWH_WIDE_ISSUE(d, d);
        }
        // tail: the last WD .. 2 WD - 1 rounds (or all of them when nr < 2 WD)
#pragma unroll
        for (int d = 0; d < 2 * WD; ++d) {
            const int r = rb + d;
            if (r < nr) SWH_WIDE_ROUND(r, d % WD, r + WD < nr);
        }
    }
#undef SWH_WIDE_ROUND
    SWH_WIDE_TRACE(1);
#undef SWH_WIDE_ISSUE

    // ---- split K (the in-launch slab hand-off of cdna_hip_programming.md, projection GEMMs item 2,
    // write-through form).  Slabs hold the accumulators in fragment order (per wave, row block
    // and column group: 64 lanes x 16 B), so every workgroup stores straight from registers —
    // no LDS tile, no barrier before the stores — drained by every wave, then one relaxed
    // agent-scope ticket.  The last arriver acquires once, issues its epilogue operands and
    // the other S - 1 slabs' pieces at once, and sums the S partials (its own from registers)
    // in fixed slab order: deterministic for any placement of the S workgroups over the XCDs.
    uint4 pre[CB][2];  // the residual epilogue's 16 columns per (row, chunk), prefetched
    if (CB == 1 && S > 1) {  // 256-row tiles never split K (wide_split): no slab code, no spills
        float *my = slabs + ((int64_t)cb * S + sidx) * (64 * NB);
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(my, 0, 64 * NB * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 1; ++j)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rsrc,
                                                       ((wid * 4 + i) * 64 + lane) * 16, 0, 16 /* sc1: write-through */);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        SWH_WIDE_TRACE(2);
        if (tid == 0) {
            const int t = __hip_atomic_fetch_add(counters + cb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag_s = (t == S - 1);
            if (t == S - 1) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
        SWH_WIDE_TRACE(3);
        if (!*flag_s) return;
        if constexpr (EPI == WEPI_RESIDUAL) {
#pragma unroll
            for (int u = 0; u < CB; ++u) {
                const int idx = tid + kWT * u, r = min(idx / (NB / 16), M - 1), j = idx % (NB / 16);
                const uint4 *sp = reinterpret_cast<const uint4 *>(res + (int64_t)r * ldy + cb * NB + 16 * j);
                pre[u][0] = sp[0];
                pre[u][1] = sp[1];
            }
        }
        const f32x4w *base = reinterpret_cast<const f32x4w *>(slabs + (int64_t)cb * S * (64 * NB));
        // every other slab's pieces in flight at once (4 x (S - 1) <= 28 per thread: the ring
        // registers are free by now): about one memory latency
        f32x4w v[4][8];
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q < S && q != sidx) {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i][q] = base[(int64_t)q * (64 * NB / 4) + (wid * 4 + i) * 64 + lane];
            }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f32x4w sum = f32x4w{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q < S) sum += q == sidx ? acc[i][0] : v[i][q];
            acc[i][0] = sum;
        }
        if (tid == 0) __hip_atomic_store(counters + cb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        SWH_WIDE_TRACE(4);
    } else if constexpr (EPI == WEPI_RESIDUAL) {
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            const int idx = tid + kWT * u, r = min(idx / (NB / 16), M - 1), j = idx % (NB / 16);
            const uint4 *sp = reinterpret_cast<const uint4 *>(res + (int64_t)r * ldy + cb * NB + 16 * j);
            pre[u][0] = sp[0];
            pre[u][1] = sp[1];
        }
    }

    // ---- this workgroup's 64 x 128 CB fp32 tile (C layout: lane holds rows 16 i + 4 kg + e,
    // column rl); the X slots it overlays are dead once every wave is past its last round
    wide_lds_barrier();
    float *tile = reinterpret_cast<float *>(lds);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) tile[(16 * i + 4 * kg + e) * LDT + wid * 16 * CB + 16 * j + rl] = acc[i][j][e];
    __syncthreads();

    // ---- epilogue
    if constexpr (EPI >= WEPI_SAMPLE) {
        // lm head + sampler (no logits): thread (row quad q, columns tid / 16 + 32 u) draws the
        // Gumbel keys of rows 4 q .. 4 q + 3 from the Philox block {col, q} exactly as
        // swh_sample_step does from the bf16 logit (EOS suppression, temperature, greedy),
        // keeps the best per row, and the workgroup's 64 bests go out as one partial each
        const int32_t step = *smp.step;
        const uint64_t seed = smp.rng[0], ctr = smp.rng[1] + (uint64_t)step;
        const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32), clo = (uint32_t)ctr, chi = (uint32_t)(ctr >> 32);
        const bool suppress = step < smp.p.min_new_tokens;
        const float temp = smp.p.temperature;
        const int q = tid & 15;
        float bk[4] = {kNegInf, kNegInf, kNegInf, kNegInf};
        int32_t bi[4] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
        float sc[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) sc[e] = NM == 2 ? rstd_s[4 * q + e] : 1.f;
        for (int c = tid >> 4; c < NB; c += kWT / 16) {
            const int col = cb * NB + c;
            float mask_add = 0.f;
            if (suppress) {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (e < smp.p.n_eos && col == smp.p.eos_ids[e]) mask_add = kNegInf;
            }
            U4 rw{0u, 0u, 0u, 0u};
            if (!smp.p.greedy) rw = philox4x32_10(U4{(uint32_t)col, (uint32_t)q, clo, chi}, k0, k1);
            const uint32_t wd[4] = {rw.x, rw.y, rw.z, rw.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float z = round_bf16(tile[(4 * q + e) * LDT + c] * sc[e]);  // the bf16 logit
                if constexpr (EPI == WEPI_SAMPLE_T) z = z / temp;
                float key = smp.p.greedy ? z : z + gumbel_from_bits(wd[e]);
                key += mask_add;
                const bool better = (key > bk[e]) | ((key == bk[e]) & (col < bi[e]));
                bk[e] = better ? key : bk[e];
                bi[e] = better ? col : bi[e];
            }
        }
        // the 4 lanes of a wave with this quad, then the waves through LDS (the tile is read)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int o = 16; o < 64; o <<= 1) {
                const float k2 = __shfl_xor(bk[e], o);
                const int32_t c2 = __shfl_xor(bi[e], o);
                if (k2 > bk[e] || (k2 == bk[e] && (uint32_t)c2 < (uint32_t)bi[e])) {
                    bk[e] = k2;
                    bi[e] = c2;
                }
            }
        __syncthreads();
        LmPart *wpart = reinterpret_cast<LmPart *>(lds);  // [W][64]
        if (lane < 16) {
#pragma unroll
            for (int e = 0; e < 4; ++e) wpart[wid * 64 + 4 * q + e] = LmPart{bk[e], bi[e]};
        }
        __syncthreads();
        if (tid < 64 && tid < M) {
            LmPart b = wpart[tid];
            for (int v = 1; v < W; ++v) {
                const LmPart o = wpart[v * 64 + tid];
                if (o.key > b.key || (o.key == b.key && (uint32_t)o.idx < (uint32_t)b.idx)) b = o;
            }
            smp.part[(int64_t)tid * smp.pstride + cb] = b;
        }
    } else if constexpr (EPI == WEPI_SILU) {
        // 64 rows x 8 groups of 8 output columns: tile columns 16 g + c (gate) and 16 g + 8 + c (up)
        for (int idx = tid; idx < 64 * (NB / 16); idx += kWT) {
            const int r = idx / (NB / 16), g = idx % (NB / 16);
            if (r >= M) continue;
            const float sc = NM == 2 ? rstd_s[r] : 1.f;
            float o[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float gv = round_bf16(tile[r * LDT + 16 * g + c] * sc);
                const float uv = round_bf16(tile[r * LDT + 16 * g + 8 + c] * sc);
                o[c] = round_bf16(gv / (1.f + expf(-gv))) * uv;
            }
            *reinterpret_cast<uint4 *>(y + (int64_t)r * ldy + cb * (NB / 2) + 8 * g) = pack8w(o);
        }
    } else if constexpr (EPI == WEPI_RESIDUAL) {
        // 64 rows x 8 chunks of 16 columns: s = bf16(s + bf16(acc)), chunk sum of squares of the new s
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            const int idx = tid + kWT * u, r = idx / (NB / 16), j = idx % (NB / 16);
            if (r >= M) continue;
            uint4 *sp = reinterpret_cast<uint4 *>(res + (int64_t)r * ldy + cb * NB + 16 * j);
            float a[16], nv[16];
            unpack16<SWH_BF16>(pre[u][0], a);
            unpack16<SWH_BF16>(pre[u][1], a + 8);
            float ss = 0.f;
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                nv[c] = round_bf16(a[c] + round_bf16(tile[r * LDT + 16 * j + c]));
                ss = fmaf(nv[c], nv[c], ss);
            }
            sp[0] = pack8w(nv);
            sp[1] = pack8w(nv + 8);
            if (ss_out) ss_out[(int64_t)r * (N / 16) + cb * (NB / 16) + j] = ss;
        }
    } else {
        // 64 rows x 16 groups of 8 columns
        for (int idx = tid; idx < 64 * (NB / 8); idx += kWT) {
            const int r = idx / (NB / 8), j = idx % (NB / 8);
            if (r >= M) continue;
            const float sc = NM == 2 ? rstd_s[r] : 1.f;
            const int col = cb * NB + 8 * j;
            float v[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = tile[r * LDT + 8 * j + c] * sc;
            if constexpr (BIAS) {
                float b[8];
                unpack16<SWH_BF16>(*reinterpret_cast<const uint4 *>(bias + col), b);
#pragma unroll
                for (int c = 0; c < 8; ++c) v[c] += b[c];
            }
            *reinterpret_cast<uint4 *>(y + (int64_t)r * ldy + col) = pack8w(v);
        }
    }
    SWH_WIDE_TRACE(5);
}

// K split: about one workgroup per CU, at most smax (the launch policy's wide_smax, 1..8:
// the last arriver reads S x 32 KB of slabs and its reduction holds up to 8 per piece)
int wide_split(int64_t ncb, int64_t K, int smax) {
    const int64_t nr = K / kWKC;
    int64_t s = (cu_count() + ncb / 2) / ncb;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    if (s > nr) s = nr;
    return (int)s;
}

// 16-row weight groups per wave: 2 when the 256-row tiles alone fill the CUs (no K split:
// the Llama-3-8B lm head, 4.57 -> 4.96 TB/s), where halving the X bytes per weight byte
// pays; with a split (gate/up: 112 tiles x 2) the hand-off cost more (58 -> 68 us), so
// 256-row tiles never split K.  The launch policy's wide_cb = 1 / 2 forces one (A/B).
int wide_cb(int64_t wcols, int64_t K, const swh_launch_policy &pol) {
    const bool two_ok = wcols % WGeo<2>::NB == 0;
    if (pol.wide_cb == 1 || !two_ok) return 1;
    if (pol.wide_cb == 2) return 2;
    return wide_split(wcols / WGeo<2>::NB, K, pol.wide_smax) == 1 ? 2 : 1;
}

// Waves per 128-row-class workgroup (16 W weight rows).  Where 8-wave tiles need no K
// split, the W in 8, 7, 6 dividing wcols whose tiles fill whole rounds of the CUs best
// (8 on ties): Llama-3-8B gate/up, 224 tiles of 128 rows -> 256 of 112, 48.1 -> 44.2 us.
// A split shape keeps 8 (qkv as 64 x 4 splits of 96 rows instead of 48 x 5: 17.4 ->
// 18.1 us; profiles/r5_waves_graph.log).  The launch policy's wide_waves forces one
// where it divides wcols (A/B).
int wide_waves(int64_t wcols, int64_t K, const swh_launch_policy &pol) {
    if (pol.wide_waves) return wcols % (16 * pol.wide_waves) == 0 ? pol.wide_waves : kWW;
    if (wcols % (16 * kWW) == 0 && wide_split(wcols / (16 * kWW), K, pol.wide_smax) > 1) return kWW;
    int best = kWW;
    double bu = -1.0;
    const int64_t cus = cu_count();
    for (int w : {8, 7, 6}) {
        if (wcols % (16 * w)) continue;
        const int64_t ncb = wcols / (16 * w);
        if (wide_split(ncb, K, pol.wide_smax) > 1) continue;
        const double u = (double)ncb / (double)(((ncb + cus - 1) / cus) * cus);
        if (u > bu + 1e-9) {
            bu = u;
            best = w;
        }
    }
    return best;
}

template <int EPI, int NM, bool BIAS, bool PACKED, int CB, int W>
int launch_wide(dim3 grid, hipStream_t st, const uint16_t *x, const uint16_t *w, int M, int N, int K, float eps,
                const float *ss_in, const uint16_t *bias, uint16_t *res, float *ss_out, uint16_t *y, int ldy,
                float *slabs, int *counters, const WSample &smp = WSample{}) {
    if (!lds_opt_in<&wide_gemm_kernel<EPI, NM, BIAS, PACKED, CB, W>>()) return SWH_E_LAUNCH;  // > 64 KB LDS
    wide_gemm_kernel<EPI, NM, BIAS, PACKED, CB, W><<<grid, WGeo<CB, W>::T, WGeo<CB, W>::LDS, st>>>(
        x, w, M, N, K, eps, ss_in, bias, res, ss_out, y, ldy, slabs, counters, smp);
    return launch_status();
}

}  // namespace

// wide tiles only: a narrow output (Qwen2.5-0.5B down, N 896) stays on decode_gemm
bool wide_gemm_eligible(int64_t M, int64_t N, int64_t K, int32_t silu) {
    const int64_t wcols = silu ? 2 * N : N;
    return M > 0 && M <= 64 && K % kWKC == 0 && K >= kWKC && wcols % kWNB == 0 && wcols >= 1024 && N % 16 == 0 &&
           wcols / kWNB <= 65535 && K < (1 << 29);
}

// Bytes of fp32 slabs the split-K reduction needs (0 when the shape is not eligible or S == 1).
int64_t wide_gemm_slab_bytes(int64_t M, int64_t N, int64_t K, int32_t silu) {
    if (!wide_gemm_eligible(M, N, K, silu)) return 0;
    // 16 W-row tiles (CB 1, the only ones that split) at the largest split the policy allows
    const int64_t wcols = silu ? 2 * N : N;
    int64_t most = 0;
    for (int w : {8, 7, 6}) {
        if (wcols % (16 * w)) continue;
        const int s = wide_split(wcols / (16 * w), K, 8);
        const int64_t b = s > 1 ? wcols * s * 64 * (int64_t)sizeof(float) : 0;
        most = b > most ? b : most;
    }
    return most;
}

template <bool P, int CB, int WV>
int dispatch_wide(dim3 grid, hipStream_t st, const uint16_t *X, const uint16_t *W, int m, int n, int k, float eps,
                  const float *ss_in, const uint16_t *B, uint16_t *R, float *ss_out, uint16_t *Y, int ld, float *slabs,
                  int *ctr, bool silu) {
#define SWH_WL(E, NMV, BI) launch_wide<E, NMV, BI, P, CB, WV>(grid, st, X, W, m, n, k, eps, ss_in, B, R, ss_out, Y, ld, slabs, ctr)
    if (silu) return ss_in ? SWH_WL(WEPI_SILU, 2, false) : SWH_WL(WEPI_SILU, 0, false);
    if (R) return SWH_WL(WEPI_RESIDUAL, 0, false);
    if (B) return ss_in ? SWH_WL(WEPI_PLAIN, 2, true) : SWH_WL(WEPI_PLAIN, 0, true);
    return ss_in ? SWH_WL(WEPI_PLAIN, 2, false) : SWH_WL(WEPI_PLAIN, 0, false);
#undef SWH_WL
}

// 1 = not eligible (the caller uses decode_gemm), else a SWH status.  packed: w is in
// wide_pack's fragment order (the same for either tiling).
int wide_gemm(const void *x, const void *w, int64_t M, int64_t N, int64_t K, float eps, const float *ss_in,
              const void *bias, void *residual, int32_t silu, void *y, int64_t ldy, float *ss_out, void *workspace,
              int64_t workspace_bytes, int64_t counter_bytes, int32_t packed, hipStream_t st) {
    if (!wide_gemm_eligible(M, N, K, silu)) return 1;
    const int64_t wcols = silu ? 2 * N : N;
    const swh_launch_policy pol = launch_policy();
    const auto *X = static_cast<const uint16_t *>(x);
    const auto *W = static_cast<const uint16_t *>(w);
    const auto *B = static_cast<const uint16_t *>(bias);
    auto *R = static_cast<uint16_t *>(residual);
    auto *Y = static_cast<uint16_t *>(y);
    const int m = (int)M, n = (int)N, k = (int)K, ld = (int)ldy;
    const int cb = wide_cb(wcols, K, pol);
    const int wv = cb == 1 ? wide_waves(wcols, K, pol) : kWW;
    const int64_t nb = 16 * (int64_t)wv * cb, ncb = wcols / nb;
    const int s = cb == 1 ? wide_split(ncb, K, pol.wide_smax) : 1;
    if (ncb * (int64_t)sizeof(int) > counter_bytes) return 1;
    float *slabs = nullptr;
    if (s > 1) {
        if (!workspace || workspace_bytes < counter_bytes + ncb * s * 64 * nb * (int64_t)sizeof(float)) return 1;
        slabs = reinterpret_cast<float *>(static_cast<char *>(workspace) + counter_bytes);
    }
    int *ctr = static_cast<int *>(workspace);
    const dim3 grid((unsigned)ncb, (unsigned)s);
#define SWH_WD(PK, CBV, WVV) dispatch_wide<PK, CBV, WVV>(grid, st, X, W, m, n, k, eps, ss_in, B, R, ss_out, Y, ld, slabs, ctr, silu)
    if (cb == 2) return packed ? SWH_WD(true, 2, 8) : SWH_WD(false, 2, 8);
    if (wv == 7) return packed ? SWH_WD(true, 1, 7) : SWH_WD(false, 1, 7);
    if (wv == 6) return packed ? SWH_WD(true, 1, 6) : SWH_WD(false, 1, 6);
    return packed ? SWH_WD(true, 1, 8) : SWH_WD(false, 1, 8);
#undef SWH_WD
}

// lm head + unfiltered sampler over a wide_pack'ed weight [V, K] (folded norm: ss_in row
// scale), 256-row tiles without a K split: one LmPart per (row, tile) into part, *pstride =
// V / 256 partials per row for the finalize.  1 = not served (the caller takes logits +
// swh_sample_step), else a SWH status.
int wide_lm_sample(const void *x, const void *w, int64_t M, int64_t V, int64_t K, float eps, const float *ss_in,
                   const swh_sample_params &p, const uint64_t *rng, const int32_t *step, LmPart *part, int *pstride,
                   hipStream_t st) {
    if (!wide_gemm_eligible(M, V, K, 0) || V % WGeo<2>::NB) return 1;
    const int ncb = (int)(V / WGeo<2>::NB);
    WSample smp{p, rng, step, part, ncb};
    *pstride = ncb;
    const dim3 grid((unsigned)ncb, 1u);
    const auto *X = static_cast<const uint16_t *>(x);
    const auto *Wt = static_cast<const uint16_t *>(w);
    const int m = (int)M, n = (int)V, k = (int)K;
    const bool tdiv = !p.greedy && p.temperature != 1.0f;
#define SWH_WS(E, NMV) launch_wide<E, NMV, false, true, 2, kWW>(grid, st, X, Wt, m, n, k, eps, ss_in, nullptr, nullptr, \
                                                              nullptr, nullptr, 0, nullptr, nullptr, smp)
    if (ss_in) return tdiv ? SWH_WS(WEPI_SAMPLE_T, 2) : SWH_WS(WEPI_SAMPLE, 2);
    return tdiv ? SWH_WS(WEPI_SAMPLE_T, 0) : SWH_WS(WEPI_SAMPLE, 0);
#undef SWH_WS
}

namespace {

// Fragment order of a [wcols, K] weight (wcols = 2N with the SiLU pairing):
//   dst[((((g * nr + q) * 4 + s) * 4 + kg) * 16 + rl) * 8 + e] = W'[row(16 g + rl)][128 q + 32 s + 8 kg + e]
// g = 16-row group in tile order (SiLU tiles: lanes 0-7 gate rows, 8-15 the matching up
// rows), q = 128-k round, s = k-step, (kg, rl) = the MFMA B-fragment lane.  W' = W, or the
// folded RMSNorm weight bf16(W * w_norm) (swh_fold_norm's product) when norm_w is given.
// One 16-B piece per thread, grid-stride; the stores are contiguous.
__global__ __launch_bounds__(256) void wide_pack_kernel(const uint16_t *__restrict__ src,
                                                        const uint16_t *__restrict__ nw, int64_t N, int64_t K,
                                                        int silu, uint16_t *__restrict__ dst, int64_t npieces) {
    const int64_t nr = K / kWKC;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npieces; p += (int64_t)gridDim.x * blockDim.x) {
        const int rl = (int)(p & 15), kg = (int)((p >> 4) & 3), s = (int)((p >> 6) & 3);
        const int64_t rest = p >> 8, q = rest % nr, g = rest / nr;
        const int64_t t = g * 16 + rl;
        const int64_t row = silu ? ((t & 15) < 8 ? (t >> 4) * 8 + (t & 7) : N + (t >> 4) * 8 + (t & 7)) : t;
        const int64_t k0 = q * kWKC + 32 * s + 8 * kg;
        uint4 v = *reinterpret_cast<const uint4 *>(src + row * K + k0);
        if (nw) {
            float a[8], b[8];
            unpack16<SWH_BF16>(v, a);
            unpack16<SWH_BF16>(*reinterpret_cast<const uint4 *>(nw + k0), b);
            uint32_t o[4];
#pragma unroll
            for (int c = 0; c < 4; ++c)
                o[c] = (uint32_t)f32_to_bf16_bits(a[2 * c] * b[2 * c]) |
                       ((uint32_t)f32_to_bf16_bits(a[2 * c + 1] * b[2 * c + 1]) << 16);
            v = uint4{o[0], o[1], o[2], o[3]};
        }
        *reinterpret_cast<uint4 *>(dst + p * 8) = v;
    }
}

}  // namespace

// the same fragment order for any 16-row group count (decode_gemm / xstream with fw)
int frag_pack(const void *src, const void *norm_w, int64_t N, int64_t K, int32_t silu, void *dst, hipStream_t st) {
    const int64_t npieces = (silu ? 2 * N : N) * K / 8;
    const int64_t grid = (npieces + 255) / 256 < 8192 ? (npieces + 255) / 256 : 8192;
    wide_pack_kernel<<<dim3((unsigned)grid), 256, 0, st>>>(static_cast<const uint16_t *>(src),
                                                             static_cast<const uint16_t *>(norm_w), N, K, silu,
                                                             static_cast<uint16_t *>(dst), npieces);
    return launch_status();
}

int wide_pack(const void *src, const void *norm_w, int64_t N, int64_t K, int32_t silu, void *dst, hipStream_t st) {
    if (!wide_gemm_eligible(1, N, K, silu)) return SWH_E_ARG;
    const int64_t npieces = (silu ? 2 * N : N) * K / 8;
    const int64_t grid = (npieces + 255) / 256 < 8192 ? (npieces + 255) / 256 : 8192;
    wide_pack_kernel<<<dim3((unsigned)grid), 256, 0, st>>>(static_cast<const uint16_t *>(src),
                                                             static_cast<const uint16_t *>(norm_w), N, K, silu,
                                                             static_cast<uint16_t *>(dst), npieces);
    return launch_status();
}

#ifdef SWH_WIDE_TRACE_ON
extern "C" int swh_wide_probe_set_trace(unsigned long long *p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_wide_trace), &p, sizeof(p)) == hipSuccess ? 0 : -2;
}
#endif

}  // namespace swh
