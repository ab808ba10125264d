// Library identity, status strings, and the library's only host-side state:
// per-device facts (call_once per device) and the explicit launch policy of the
// calling thread (thread_local: no process-wide mutable state).
#include "common.hpp"

namespace swh {

int cu_count() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
    static std::once_flag once[kMaxDevices];
    static int cus[kMaxDevices];
    std::call_once(once[dev], [dev] {
        int n = 0;
        cus[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
    });
    return cus[dev];
}

bool lds_opt_in_once(const void *kernel, std::once_flag *once, bool *ok) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return false;
    std::call_once(once[dev], [&] {
        ok[dev] = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxDynLds) == hipSuccess;
    });
    return ok[dev];
}

namespace {
swh_launch_policy default_policy() {
    swh_launch_policy p{};
    p.wide_kmin = 2048;
    p.wide_gemm = 1;
    p.wide_smax = 8;
    p.xstream = 1;
    p.lm_ring14 = 1;
    p.filt_wgs = 1024;
    p.attn_pair = 1;
    return p;
}
// each host thread holds its own policy (the defaults until it sets one), so two
// callers in one process cannot change each other's geometry or output bits
thread_local swh_launch_policy t_policy = default_policy();

bool in(int32_t v, std::initializer_list<int32_t> ok) {
    for (int32_t o : ok)
        if (v == o) return true;
    return false;
}
}  // namespace

swh_launch_policy launch_policy() { return t_policy; }

}  // namespace swh

using namespace swh;

extern "C" int swh_launch_policy_default(swh_launch_policy *out) {
    if (!out) return SWH_E_ARG;
    *out = default_policy();
    return SWH_OK;
}

extern "C" int swh_get_launch_policy(swh_launch_policy *out) {
    if (!out) return SWH_E_ARG;
    *out = launch_policy();
    return SWH_OK;
}

extern "C" int swh_set_launch_policy(const swh_launch_policy *p) {
    if (!p) return SWH_E_ARG;
    const bool geo_auto = p->gemm_ms == 0;
    if (p->wide_kmin < 32 || !in(p->wide_gemm, {0, 1}) || p->wide_smax < 1 || p->wide_smax > 8 ||
        !in(p->wide_cb, {0, 1, 2}) || !in(p->gemm_ms, {0, 1, 2, 4}) ||
        (geo_auto ? (p->gemm_cb || p->gemm_s || p->gemm_persist || p->gemm_wn)
                  : (!in(p->gemm_cb, {1, 2, 4}) || p->gemm_s < 1 || p->gemm_s > 8 || !in(p->gemm_persist, {0, 1}) ||
                     !in(p->gemm_wn, {1, 2, 4}))) ||
        !in(p->gemm_tile, {0, 1}) || !in(p->gemm_nw, {0, 4, 8, 16}) || !in(p->xstream, {0, 1}) ||
        !in(p->lm_ring14, {0, 1}) || p->filt_wgs < 64 || p->filt_wgs > 65536 || !in(p->wide_waves, {0, 6, 7, 8}) ||
        !in(p->attn_pair, {0, 1}))
        return SWH_E_ARG;
    t_policy = *p;
    return SWH_OK;
}

extern "C" const char *swh_version(void) { return "swh_trl_amd 0.1.0 (gfx950)"; }

extern "C" const char *swh_status_string(int status) {
    switch (status) {
    case SWH_OK: return "ok";
    case SWH_E_ARG: return "invalid argument";
    case SWH_E_LAUNCH: return "kernel launch failed";
    case SWH_E_DTYPE: return "unsupported dtype";
    default: return "unknown status";
    }
}
