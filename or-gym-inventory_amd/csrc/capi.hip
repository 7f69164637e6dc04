// C ABI of libinvsim (include/invsim.h): handle lifetime, HBM state arena,
// spec validation (the reference's assert checks), and kernel launches.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/invsim.h"
#include "kernels.hpp"

using namespace invsim;

namespace {

thread_local std::string g_last_error;

struct Field {
    std::string name;
    int64_t offset;   // bytes from arena start
    int32_t elem;     // element bytes
    int32_t rows;     // rows, or record width
    int32_t kind;     // 0: [rows][Npad]; 1: record [Npad][rows]; 2: other (opaque)
};

}  // namespace

namespace invsim {
int net_spec_match(const invsim_netinvmgmt_spec &h);   // netspec.hip
#ifdef INVSIM_PTRS_STATS
hipError_t ptrs_stats_nv(unsigned long long *out, bool clear);
hipError_t ptrs_stats_nv_ph(unsigned long long *out, bool clear);
hipError_t ptrs_stats_im(unsigned long long *out, bool clear);
hipError_t ptrs_stats_im_ph(unsigned long long *out, bool clear);
hipError_t ptrs_stats_netspec(unsigned long long *out, bool clear);
hipError_t ptrs_stats_net(unsigned long long *out, bool clear);
#endif
}

struct invsim_handle {
    int32_t family = 0;
    int32_t device = 0;
    int64_t N = 0, Npad = 0;
    int32_t obs_dim = 0, act_dim = 0, demand_dim = 1;
    char *arena = nullptr;      // state (get/set_state blob)
    int64_t arena_bytes = 0;
    char *tables = nullptr;     // read-only tables (not part of the state blob)
    void *scratch = nullptr;    // caches derived from the state (not part of the blob)
    bool la_valid = false;      // demand lookahead cache (Im/NvParams::ahead) is valid
    int la_slot = 0;            //   ... with this current slot
    std::vector<Field> fields;
    Common cm{};
    NvParams nv{};
    ImParams im{};
    NetParams net{};
    int32_t im_m1 = 0;
    bool im_backlog = false;
    int32_t net_spec = 0;     // NET_SPEC_*: compile-time specialised kernel for this graph
    // lock-step period tracking (see kernels.hpp next_period)
    bool t_known = true;
    int32_t t_cur = 0;
    int32_t horizon = 0;
    bool past_ok = false;     // Newsvendor keeps stepping past step_limit with autoreset off
    // demand stream (invsim_set_demand_stream): numpy PCG64 (parity) or the fast
    // counter-based Philox stream, whose launch-step counter lives here and in
    // the state blob ("philox_step")
    int32_t demand_stream = INVSIM_DEMAND_NUMPY;
    uint64_t ph_step = 0;
    int64_t o_phstep = 0;
    bool ph_from_blob = false;  // set_state loaded the blob: its philox_step is the counter
    // graph capture (invsim_capture_begin / _end): the host-side position at
    // begin, put back at end, and the env steps the captured calls enqueue
    bool capturing = false;
    bool cap_t_known = true, cap_la_valid = false;
    int32_t cap_t_cur = 0;
    int cap_la_slot = 0;
    int64_t cap_steps = 0;
    std::string err;
};

namespace {

// roctx range around an ABI call (SURVEY §5 tracing: step / rollout / reset
// show up as named ranges under `rocprofv3 --marker-trace`; a no-op call when
// no profiler is attached).  roctx is opened with dlopen at the first call, so
// libinvsim.so has no load-time dependency on it; without it ranges are no-ops.
struct Roctx {
    int (*push)(const char *) = nullptr;
    int (*pop)() = nullptr;
    Roctx() {
        void *so = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!so) so = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!so) return;
        push = reinterpret_cast<int (*)(const char *)>(dlsym(so, "roctxRangePushA"));
        pop = reinterpret_cast<int (*)()>(dlsym(so, "roctxRangePop"));
        if (!push || !pop) push = nullptr, pop = nullptr;
    }
};

const Roctx &roctx() {
    static const Roctx r;
    return r;
}

struct TraceRange {
    explicit TraceRange(const char *name) {
        if (roctx().push) roctx().push(name);
    }
    ~TraceRange() {
        if (roctx().pop) roctx().pop();
    }
};

struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int fail(invsim_handle *h, int code, const std::string &msg) {
    if (h) h->err = msg;
    g_last_error = msg;
    return code;
}

int hip_fail(invsim_handle *h, hipError_t e, const char *what) {
    return fail(h, INVSIM_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

// Calls that synchronise with the host cannot be recorded into a graph.
int refuse_in_capture(invsim_handle *h, const char *what) {
    if (!h->capturing) return INVSIM_OK;
    return fail(h, INVSIM_EINVAL, std::string(what) + " synchronises with the host and cannot be captured "
                                                      "(between invsim_capture_begin and invsim_capture_end)");
}

// A launching call on a stream that is being captured must be inside the
// capture bracket: otherwise the host-side position advances while the device
// state does not (nothing runs until the graph is replayed).
int capture_check(invsim_handle *h, hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) {
        (void)hipGetLastError();   // e.g. the legacy stream while another one captures: not ours to record
        st = hipStreamCaptureStatusNone;
    }
    if (st == hipStreamCaptureStatusActive && !h->capturing)
        return fail(h, INVSIM_EINVAL, "this stream is being captured into a graph: bracket the capture with "
                                      "invsim_capture_begin / invsim_capture_end");
    return INVSIM_OK;
}

// Lay out named SoA fields (rows x Npad elements each, 256-byte aligned).
struct Layout {
    std::vector<Field> f;
    int64_t bytes = 0;
    int64_t add(const char *name, int32_t elem, int32_t rows, int64_t npad, int32_t kind = 0) {
        bytes = (bytes + 255) / 256 * 256;
        Field x{name, bytes, elem, rows, kind};
        f.push_back(x);
        bytes += (int64_t)elem * rows * npad;
        return x.offset;
    }
};

template <typename T>
T *at(invsim_handle *h, int64_t off) {
    return reinterpret_cast<T *>(h->arena + off);
}

int alloc_arena(invsim_handle *h, const Layout &lay) {
    h->fields = lay.f;
    h->arena_bytes = std::max<int64_t>(lay.bytes, 256);
    hipError_t e = hipMalloc(&h->arena, (size_t)h->arena_bytes);
    if (e != hipSuccess) return fail(h, INVSIM_ENOMEM, std::string("hipMalloc(state): ") + hipGetErrorString(e));
    e = hipMemset(h->arena, 0, (size_t)h->arena_bytes);
    if (e != hipSuccess) return hip_fail(h, e, "hipMemset(state)");
    return INVSIM_OK;
}

int common_fields(invsim_handle *h, Layout &lay, int64_t &o_rng, int64_t &o_period, int64_t &o_status) {
    o_rng = lay.add("rng", 8, 4, h->Npad);   // rows: state_hi, state_lo, inc_hi, inc_lo
    o_period = lay.add("period", 4, 1, h->Npad);
    o_status = lay.add("status", 4, 1, 1);
    h->o_phstep = lay.add("philox_step", 8, 1, 1);
    return 0;
}

// The A/B launch switches (kernels.hpp Knobs), read from the environment once,
// here, when a handle is created: the only environment reads of the library.
// A switch is "0" or "1" exactly; anything else (unset, empty, "false", "on")
// keeps the default.
bool env_flag(const char *name, bool dflt) {
    const char *v = std::getenv(name);
    if (!v || (v[0] != '0' && v[0] != '1') || v[1]) return dflt;
    return v[0] == '1';
}

Knobs read_knobs() {
    Knobs k;
    k.im_split = env_flag("INVSIM_IM_SPLIT", k.im_split);
    k.im_la_last = env_flag("INVSIM_IM_LA_LAST", k.im_la_last);
    k.im_roll = env_flag("INVSIM_IM_ROLL", k.im_roll);
    k.im_pol_roll = env_flag("INVSIM_IM_POL_ROLL", k.im_pol_roll);
    k.im_ahead = env_flag("INVSIM_IM_AHEAD", k.im_ahead);
    if (const char *v = std::getenv("INVSIM_IM_ROLL3O_G2"); v && (v[0] == '0' || v[0] == '1'))
        k.im_roll3o_g2 = (int8_t)(v[0] - '0');
    auto count = [](const char *name, int64_t &dst) {   // a decimal count, else the default
        if (const char *v = std::getenv(name); v && v[0]) {
            char *end = nullptr;
            const long long x = std::strtoll(v, &end, 10);
            if (end && !*end && x >= 0) dst = (int64_t)x;
        }
    };
    count("INVSIM_IM_ROLL3O_MAX_N", k.im_roll3o_max_n);
    count("INVSIM_IM_ROLL_SUB", k.im_roll_sub);
    count("INVSIM_NET_ROLLQ_MAX_N", k.net_rollq_max_n);
    count("INVSIM_NET_ROLL4_MAX_N", k.net_roll4_max_n);
    k.nv_xcd = env_flag("INVSIM_NV_XCD", k.nv_xcd);
    k.nv_roll = env_flag("INVSIM_NV_ROLL", k.nv_roll);
    k.nv_pol_roll = env_flag("INVSIM_NV_POL_ROLL", k.nv_pol_roll);
    k.nv_ahead = env_flag("INVSIM_NV_AHEAD", k.nv_ahead);
    k.net_roll = env_flag("INVSIM_NET_ROLL", k.net_roll);
    k.net_roll3 = env_flag("INVSIM_NET_ROLL3", k.net_roll3);
    k.net_split = env_flag("INVSIM_NET_SPLIT", k.net_split);
    k.net_pol_roll = env_flag("INVSIM_NET_POL_ROLL", k.net_pol_roll);
    k.net_ahead = env_flag("INVSIM_NET_AHEAD", k.net_ahead);
    k.net_generic = env_flag("INVSIM_NET_GENERIC", k.net_generic);
    return k;
}

void bind_common(invsim_handle *h, int64_t o_rng, int64_t o_period, int64_t o_status, int32_t ar) {
    Common &c = h->cm;
    c.kn = read_knobs();
    c.N = h->N;
    c.Npad = h->Npad;
    c.autoreset = ar;
    uint64_t *r = at<uint64_t>(h, o_rng);
    c.rng.hi = r;
    c.rng.lo = r + h->Npad;
    c.rng.inc_hi = r + 2 * h->Npad;
    c.rng.inc_lo = r + 3 * h->Npad;
    c.period = at<int32_t>(h, o_period);
    c.status = at<uint32_t>(h, o_status);
    c.info_demand = nullptr;
    c.u32buf = nullptr;
    c.info_rec = nullptr;
}

// "done" marker: period = horizon, so NEXT_STEP autoreset resets on first step
int init_period(invsim_handle *h, int32_t horizon) {
    h->horizon = horizon;
    h->t_known = true;
    h->t_cur = horizon;  // "done": the first NEXT_STEP step resets
    std::vector<int32_t> v((size_t)h->Npad, horizon);
    hipError_t e = hipMemcpy(h->cm.period, v.data(), sizeof(int32_t) * h->Npad, hipMemcpyHostToDevice);
    return e == hipSuccess ? INVSIM_OK : hip_fail(h, e, "hipMemcpy(period)");
}

int upload_tables(invsim_handle *h, const std::vector<char> &blob) {
    if (blob.empty()) return INVSIM_OK;
    hipError_t e = hipMalloc(&h->tables, blob.size());
    if (e != hipSuccess) return fail(h, INVSIM_ENOMEM, "hipMalloc(tables)");
    e = hipMemcpy(h->tables, blob.data(), blob.size(), hipMemcpyHostToDevice);
    return e == hipSuccess ? INVSIM_OK : hip_fail(h, e, "hipMemcpy(tables)");
}

// host-side packer for read-only tables
struct Blob {
    std::vector<char> b;
    template <typename T>
    int64_t put(const T *p, size_t n) {
        size_t off = (b.size() + 15) / 16 * 16;
        b.resize(off + std::max<size_t>(n, 1) * sizeof(T), 0);
        if (p && n) std::memcpy(b.data() + off, p, n * sizeof(T));
        return (int64_t)off;
    }
};

template <typename T>
const T *tab(invsim_handle *h, int64_t off) {
    return reinterpret_cast<const T *>(h->tables + off);
}

bool valid_autoreset(int32_t m) { return m >= 0 && m <= 2; }

int finish_create(invsim_handle *h, invsim_handle **out, int rc) {
    if (rc != INVSIM_OK) {
        g_last_error = h->err;
        invsim_destroy(h);
        *out = nullptr;
        return rc;
    }
    *out = h;
    return INVSIM_OK;
}

int64_t pad_n(int64_t n) { return std::max<int64_t>(256, (n + 255) / 256 * 256); }

// Host table of PTRS's right-hand side  -lam + k*log(lam) - loggam(k+1)  for the
// k that occur in practice (lam +- 12 sd), evaluated with the host libm exactly as
// numpy evaluates it (distributions.c random_poisson_ptrs).  The device looks it
// up instead of computing a log-gamma per rejection test; k outside falls back.
void rhs_table(PtrsConst &c, std::vector<double> &tab) {
    c.k0 = 0;
    c.nk = 0;
    c.toff = (int32_t)tab.size();
    if (!(c.lam >= 10) || c.lam > 1e8) return;
    const double sd = std::sqrt(c.lam);
    int64_t k0 = std::max<int64_t>(0, (int64_t)std::floor(c.lam - 12 * sd - 10));
    const int64_t k1 = (int64_t)std::ceil(c.lam + 12 * sd + 40);
    int64_t n = k1 - k0;
    if (n > RHS_LDS_MAX) {      // keep the central RHS_LDS_MAX entries (the rest: device)
        k0 = std::max<int64_t>(0, (int64_t)std::floor(c.lam) - RHS_LDS_MAX / 2 + 20);
        n = RHS_LDS_MAX;
    }
    for (int64_t k = k0; k < k0 + n; k++)
        tab.push_back(-c.lam + (double)k * c.loglam - np_loggam((double)(k + 1)));
    c.k0 = (int32_t)k0;
    c.nk = (int32_t)n;
}

}  // namespace

extern "C" {

int invsim_abi_version(void) { return INVSIM_ABI_VERSION; }

const char *invsim_last_error(const invsim_handle *h) {
    return h ? h->err.c_str() : g_last_error.c_str();
}

void invsim_destroy(invsim_handle *h) {
    if (!h) return;
    DeviceGuard g(h->device);
    if (h->arena) (void)hipFree(h->arena);
    if (h->tables) (void)hipFree(h->tables);
    if (h->scratch) (void)hipFree(h->scratch);
    delete h;
}

// ------------------------------------------------------------------ Newsvendor
int invsim_create_newsvendor(const invsim_newsvendor_spec *spec, int64_t n, int32_t device,
                             int32_t ar, invsim_handle **out) {
    if (!spec || !out) return fail(nullptr, INVSIM_EINVAL, "null argument");
    if (n < 0 || n > (int64_t)1 << 31) return fail(nullptr, INVSIM_EINVAL, "n_envs out of range");
    if (!valid_autoreset(ar)) return fail(nullptr, INVSIM_EINVAL, "bad autoreset mode");
    const int L = std::max(0, spec->lead_time);  // newsvendor.py:65
    if (L > 128) return fail(nullptr, INVSIM_ERANGE, "lead_time > 128 not supported");
    if (!(spec->mu_max >= 0) || spec->mu_max > 1e18)
        return fail(nullptr, INVSIM_EINVAL, "mu_max must be in [0, 1e18] (numpy poisson lam range)");
    DeviceGuard g(device);
    if (!g.ok) return fail(nullptr, INVSIM_EDEVICE, "hipSetDevice failed");
    auto *h = new invsim_handle();
    h->family = INVSIM_NEWSVENDOR;
    h->device = device;
    h->N = n;
    h->Npad = pad_n(n);
    h->obs_dim = L + 5;
    h->act_dim = 1;
    Layout lay;
    int64_t o_rng, o_per, o_st;
    common_fields(h, lay, o_rng, o_per, o_st);
    int64_t o_par = lay.add("params", 8, 5, h->Npad);
    int64_t o_pipe = lay.add("pipeline", 4, std::max(L, 1), h->Npad);
    // loggam(k + 1) for the per-env PTRS right-hand side (numpy's formula, host libm)
    Blob tb;
    std::vector<double> lg(RHS_LDS_MAX);
    for (int k = 0; k < RHS_LDS_MAX; k++) lg[k] = np_loggam((double)(k + 1));
    const int64_t t_lg = tb.put(lg.data(), lg.size());
    int rc = alloc_arena(h, lay);
    if (rc == INVSIM_OK) rc = upload_tables(h, tb.b);
    if (rc == INVSIM_OK) {
        bind_common(h, o_rng, o_per, o_st, ar);
        NvParams &p = h->nv;
        p.lgtab = tab<double>(h, t_lg);
        p.cm = h->cm;
        p.L = L;
        p.step_limit = spec->step_limit;
        p.max_inventory = spec->max_inventory;
        p.max_order = spec->max_order_quantity;
        p.p_max = spec->p_max;
        p.h_max = spec->h_max;
        p.k_max = spec->k_max;
        p.mu_max = spec->mu_max;
        p.par = at<double>(h, o_par);
        p.pipe = at<float>(h, o_pipe);
        p.ahead = nullptr;
        p.pcon = nullptr;
        {   // demand lookahead cache: 2 slots x 3 rows x Npad u64, then 6 rows of Poisson constants
            hipError_t e = hipMalloc(&h->scratch, (size_t)((2 * 3 + 6) * h->Npad * sizeof(uint64_t)));
            if (e != hipSuccess) {
                rc = fail(h, INVSIM_ENOMEM, "hipMalloc(lookahead cache)");
            } else {
                p.ahead = static_cast<uint64_t *>(h->scratch);
                p.pcon = reinterpret_cast<double *>(p.ahead + 2 * 3 * h->Npad);
            }
        }
        h->past_ok = true;
        if (rc == INVSIM_OK) rc = init_period(h, std::max(spec->step_limit, 0));
    }
    return finish_create(h, out, rc);
}

// ------------------------------------------------------------------ InvMgmt
int invsim_create_invmgmt(const invsim_invmgmt_spec *s, int64_t n, int32_t device, int32_t ar,
                          invsim_handle **out) {
    if (!s || !out) return fail(nullptr, INVSIM_EINVAL, "null argument");
    if (n < 0 || n > (int64_t)1 << 31) return fail(nullptr, INVSIM_EINVAL, "n_envs out of range");
    if (!valid_autoreset(ar)) return fail(nullptr, INVSIM_EINVAL, "bad autoreset mode");
    const int m = s->num_stages, m1 = m - 1;
    // inventory_management.py:144-167 validation
    if (m < 2) return fail(nullptr, INVSIM_EINVAL, "Minimum number of stages is 2");
    if (m1 > IM_MAX_M1) return fail(nullptr, INVSIM_ERANGE, "at most 9 stages supported");
    if (s->periods <= 0) return fail(nullptr, INVSIM_EINVAL, "Number of periods must be positive");
    if (!s->I0 || !s->unit_price || !s->unit_cost || !s->demand_cost || !s->holding_cost ||
        !s->supply_capacity || !s->lead_time)
        return fail(nullptr, INVSIM_EINVAL, "null parameter array");
    for (int i = 0; i < m1; i++) {
        if (s->I0[i] < 0) return fail(nullptr, INVSIM_EINVAL, "Initial inventory cannot be negative");
        if (s->supply_capacity[i] <= 0) return fail(nullptr, INVSIM_EINVAL, "Supply capacities must be positive");
        if (s->lead_time[i] < 0) return fail(nullptr, INVSIM_EINVAL, "Lead times cannot be negative");
        if (s->lead_time[i] > 255) return fail(nullptr, INVSIM_ERANGE, "lead time > 255 not supported");
    }
    for (int j = 0; j < m; j++) {
        if (!(s->unit_price[j] >= 0)) return fail(nullptr, INVSIM_EINVAL, "Sales prices cannot be negative");
        if (!(s->unit_cost[j] >= 0)) return fail(nullptr, INVSIM_EINVAL, "Procurement costs cannot be negative");
        if (!(s->demand_cost[j] >= 0)) return fail(nullptr, INVSIM_EINVAL, "Unfulfilled demand costs cannot be negative");
        if (!(s->holding_cost[j] >= 0)) return fail(nullptr, INVSIM_EINVAL, "Holding costs cannot be negative");
    }
    if (!(s->alpha > 0 && s->alpha <= 1)) return fail(nullptr, INVSIM_EINVAL, "alpha must be in the range (0, 1]");
    if (s->dist == 1) {
        if (!(s->mu >= 0) || s->mu > 1e18) return fail(nullptr, INVSIM_EINVAL, "poisson mu out of range");
    } else if (s->dist == 5) {
        if (!s->user_D) return fail(nullptr, INVSIM_EINVAL, "User specified demand length != num periods");
    } else if (s->dist == 2) {   // numpy Generator.binomial argument checks
        if (s->dist_n < 0) return fail(nullptr, INVSIM_EINVAL, "n < 0");
        if (!(s->dist_p >= 0 && s->dist_p <= 1)) return fail(nullptr, INVSIM_EINVAL, "p < 0, p > 1 or p is NaN");
    } else if (s->dist == 3) {   // Generator.integers(low, high + 1)
        if (s->dist_high == INT64_MAX) return fail(nullptr, INVSIM_EINVAL, "high is out of bounds for int64");
        if (s->dist_low > s->dist_high) return fail(nullptr, INVSIM_EINVAL, "low >= high");
    } else if (s->dist == 4) {   // Generator.geometric
        if (!(s->dist_p > 0 && s->dist_p <= 1)) return fail(nullptr, INVSIM_EINVAL, "p <= 0, p > 1 or p contains NaNs");
    } else {
        return fail(nullptr, INVSIM_EINVAL, "dist must be one of 1, 2, 3, 4, 5");
    }
    DeviceGuard g(device);
    if (!g.ok) return fail(nullptr, INVSIM_EDEVICE, "hipSetDevice failed");
    auto *h = new invsim_handle();
    h->family = INVSIM_INVMGMT;
    h->device = device;
    h->N = n;
    h->Npad = pad_n(n);
    int D = 0, sumL = 0;
    for (int i = 0; i < m1; i++) {
        D = std::max<int>(D, (int)s->lead_time[i]);
        sumL += (int)s->lead_time[i];
    }
    h->obs_dim = m1 * (D + 1);
    h->act_dim = m1;
    if (h->obs_dim > 320) {
        delete h;
        return fail(nullptr, INVSIM_ERANGE, "observation length (m-1)*(max(L)+1) > 320 not supported");
    }
    h->im_m1 = m1;
    h->im_backlog = s->backlog != 0;
    Layout lay;
    int64_t o_rng, o_per, o_st;
    common_fields(h, lay, o_rng, o_per, o_st);
    int64_t o_I = lay.add("I", 8, m1, h->Npad);
    int64_t o_B = lay.add("B", 8, h->im_backlog ? m : 1, h->Npad);
    int64_t o_R = lay.add("Rring", 8, std::max(sumL, 1), h->Npad);
    int64_t o_A = lay.add("alog", 8, std::max(D * m1, 1), h->Npad, 2);      // [D][Npad][m1]
    int64_t o_A32 = lay.add("alog32", 4, std::max(D * m1, 1), h->Npad, 2);  // [D][Npad][m1]
    // Generator.integers draws 32-bit halves: the bit generator's buffered half is
    // state (the dist 2-4 kernel variant carries the row; only dist 3 uses it)
    const int64_t o_U32 = (s->dist >= 2 && s->dist <= 4) ? lay.add("u32buf", 8, 1, h->Npad) : -1;
    // read-only tables: alpha**t (Python float pow == C pow), user_D
    Blob tb;
    std::vector<double> ap((size_t)s->periods);
    for (int t = 0; t < s->periods; t++) ap[t] = std::pow(s->alpha, (double)t);
    int64_t o_ap = tb.put(ap.data(), ap.size());
    std::vector<int64_t> ud((size_t)s->periods, 0);
    if (s->dist == 5) std::memcpy(ud.data(), s->user_D, sizeof(int64_t) * s->periods);
    int64_t o_ud = tb.put(ud.data(), ud.size());
    PtrsConst pc = ptrs_const(s->dist == 1 ? s->mu : 0.0);  // host libm, as numpy
    std::vector<double> rhs;
    rhs_table(pc, rhs);
    const int64_t o_rhs = tb.put(rhs.data(), rhs.size());
    int rc = alloc_arena(h, lay);
    if (rc == INVSIM_OK) rc = upload_tables(h, tb.b);
    if (rc == INVSIM_OK) {
        bind_common(h, o_rng, o_per, o_st, ar);
        if (o_U32 >= 0) h->cm.u32buf = at<uint64_t>(h, o_U32);
        ImParams &p = h->im;
        p.rhs = pc.nk > 0 ? tab<double>(h, o_rhs) : nullptr;
        p.cm = h->cm;
        if (s->dist == 2) p.nd = np_dist_binomial(s->dist_n, s->dist_p);
        if (s->dist == 3) p.nd = np_dist_integers(s->dist_low, s->dist_high);
        if (s->dist == 4) p.nd = np_dist_geometric(s->dist_p);
        p.periods = s->periods;
        p.lt_max = D;
        p.dist = s->dist;
        int off = 0;
        for (int i = 0; i < m1; i++) {
            p.L[i] = (int32_t)s->lead_time[i];
            p.ring_off[i] = off;
            off += p.L[i];
            p.c[i] = s->supply_capacity[i];
            p.I0[i] = s->I0[i];
        }
        for (int j = 0; j < m; j++) {
            p.up[j] = (double)s->unit_price[j];
            p.uc[j] = (double)s->unit_cost[j];
            p.hc[j] = (double)s->holding_cost[j];
            p.kc[j] = (double)s->demand_cost[j];
        }
        p.pc = pc;
        p.alpha_pow = tab<double>(h, o_ap);
        p.user_D = tab<int64_t>(h, o_ud);
        p.I = at<int64_t>(h, o_I);
        p.B = at<int64_t>(h, o_B);
        p.Rring = at<int64_t>(h, o_R);
        p.alog = at<int64_t>(h, o_A);
        p.alog32 = at<uint32_t>(h, o_A32);
        p.ahead = nullptr;
        if (s->dist >= 1 && s->dist <= 4) {   // demand lookahead cache: 2 slots x 4 rows x Npad u64
            hipError_t e = hipMalloc(&h->scratch, (size_t)(2 * 4 * h->Npad * sizeof(uint64_t)));
            if (e != hipSuccess) rc = fail(h, INVSIM_ENOMEM, "hipMalloc(lookahead cache)");
            else p.ahead = static_cast<uint64_t *>(h->scratch);
        }
        if (rc == INVSIM_OK) rc = init_period(h, s->periods);
    }
    return finish_create(h, out, rc);
}

// ------------------------------------------------------------------ NetInvMgmt
int invsim_create_netinvmgmt(const invsim_netinvmgmt_spec *s, int64_t n, int32_t device, int32_t ar,
                             invsim_handle **out) {
    if (!s || !out) return fail(nullptr, INVSIM_EINVAL, "null argument");
    if (n < 0 || n > (int64_t)1 << 31) return fail(nullptr, INVSIM_EINVAL, "n_envs out of range");
    if (!valid_autoreset(ar)) return fail(nullptr, INVSIM_EINVAL, "bad autoreset mode");
    const int J = s->n_main, E = s->n_reorder, RL = s->n_retail;
    if (J < 1 || E < 0 || RL < 0 || J > 64 || E > 256 || RL > 64)
        return fail(nullptr, INVSIM_ERANGE, "topology size out of supported range");
    if (s->num_periods <= 0) return fail(nullptr, INVSIM_EINVAL, "num_periods must be positive");
    if (!(s->alpha > 0 && s->alpha <= 1)) return fail(nullptr, INVSIM_EINVAL, "alpha must be in (0, 1]");
    if (!s->I0 || !s->h || !s->C || !s->o || !s->v || !s->is_factory || !s->is_retail ||
        (E && (!s->sup || !s->pur || !s->sup_is_factory || !s->L || !s->lp || !s->lg)) ||
        (RL && (!s->rl_node || !s->rl_p || !s->rl_b || !s->rl_lam || !s->rl_user)) ||
        !s->succ_ptr || !s->pred_ptr)
        return fail(nullptr, INVSIM_EINVAL, "null topology table");
    // network_management.py:197-238 validation
    for (int j = 0; j < J; j++) {
        if (!(s->I0[j] >= 0)) return fail(nullptr, INVSIM_EINVAL, "Invalid or missing I0>=0");
        if (!(s->h[j] >= 0)) return fail(nullptr, INVSIM_EINVAL, "Invalid or missing h>=0");
        if (s->is_factory[j]) {
            if (!(s->C[j] > 0)) return fail(nullptr, INVSIM_EINVAL, "Invalid or missing C>0");
            if (!(s->o[j] >= 0)) return fail(nullptr, INVSIM_EINVAL, "Invalid or missing o>=0");
            if (!(s->v[j] > 0 && s->v[j] <= 1)) return fail(nullptr, INVSIM_EINVAL, "Invalid or missing v in (0, 1]");
        }
        if (!(s->v[j] > 0)) return fail(nullptr, INVSIM_EINVAL, "yield v must be > 0");
    }
    int sumL = 0;
    for (int k = 0; k < E; k++) {
        if (s->L[k] < 0 || s->L[k] > 255) return fail(nullptr, INVSIM_ERANGE, "Invalid or missing L>=0 (max 255)");
        if (!(s->lp[k] >= 0) || !(s->lg[k] >= 0)) return fail(nullptr, INVSIM_EINVAL, "Invalid or missing p/g>=0");
        if (s->sup[k] < -1 || s->sup[k] >= J || s->pur[k] < 0 || s->pur[k] >= J)
            return fail(nullptr, INVSIM_EINVAL, "reorder link endpoint out of range");
        sumL += s->L[k];
    }
    for (int r = 0; r < RL; r++) {
        if (s->rl_node[r] < 0 || s->rl_node[r] >= J) return fail(nullptr, INVSIM_EINVAL, "retail link node out of range");
        if (!(s->rl_p[r] >= 0) || !(s->rl_b[r] >= 0)) return fail(nullptr, INVSIM_EINVAL, "Invalid or missing p/b>=0");
        const int dk = s->rl_dist ? s->rl_dist[r] : 1;
        if (!s->rl_user[r]) {
            if (dk < 1 || dk > 4) return fail(nullptr, INVSIM_EINVAL, "market sampler must be 1..4");
            if (dk == 1 && (!(s->rl_lam[r] >= 0) || s->rl_lam[r] > 1e18))
                return fail(nullptr, INVSIM_EINVAL, "poisson lam out of range");
            if (dk > 1 && (!s->rl_n || !s->rl_high || !s->rl_dp)) return fail(nullptr, INVSIM_EINVAL, "null market sampler table");
            if (dk == 2 && (s->rl_n[r] < 0 || !(s->rl_dp[r] >= 0 && s->rl_dp[r] <= 1)))
                return fail(nullptr, INVSIM_EINVAL, "binomial market needs n >= 0 and 0 <= p <= 1");
            if (dk == 3 && !(s->rl_high[r] > s->rl_n[r]))
                return fail(nullptr, INVSIM_EINVAL, "integers market: low >= high");
            if (dk == 4 && !(s->rl_dp[r] > 0 && s->rl_dp[r] <= 1))
                return fail(nullptr, INVSIM_EINVAL, "geometric market needs 0 < p <= 1");
        }
        if (s->rl_user[r] && !s->user_D) return fail(nullptr, INVSIM_EINVAL, "user_D table missing");
    }
    const int nsucc = s->succ_ptr[J], npred = s->pred_ptr[J];
    if (nsucc < 0 || npred < 0 || (nsucc && (!s->succ_kind || !s->succ_idx)) || (npred && !s->pred_idx))
        return fail(nullptr, INVSIM_EINVAL, "bad adjacency tables");
    for (int q = 0; q < nsucc; q++) {
        if (s->succ_kind[q] == 0 ? (s->succ_idx[q] < 0 || s->succ_idx[q] >= E)
                                 : (s->succ_idx[q] < 0 || s->succ_idx[q] >= RL))
            return fail(nullptr, INVSIM_EINVAL, "successor index out of range");
    }
    for (int q = 0; q < npred; q++)
        if (s->pred_idx[q] < 0 || s->pred_idx[q] >= E) return fail(nullptr, INVSIM_EINVAL, "predecessor index out of range");
    DeviceGuard g(device);
    if (!g.ok) return fail(nullptr, INVSIM_EDEVICE, "hipSetDevice failed");
    auto *h = new invsim_handle();
    h->family = INVSIM_NETINVMGMT;
    h->device = device;
    h->N = n;
    h->Npad = pad_n(n);
    h->obs_dim = RL + J + sumL;
    h->act_dim = E;
    h->demand_dim = std::max(RL, 1);
    Layout lay;
    int64_t o_rng, o_per, o_st;
    common_fields(h, lay, o_rng, o_per, o_st);
    int64_t o_X = lay.add("X", 8, J, h->Npad);
    int64_t o_U = lay.add("U", 8, std::max(RL, 1), h->Npad);
    int64_t o_Y = lay.add("Y", 8, std::max(E, 1), h->Npad);
    int64_t o_R = lay.add("Rring", 8, std::max(sumL, 1), h->Npad);
    bool any_int = false, any_npd = false;
    std::vector<int32_t> rdist((size_t)std::max(RL, 1), 1);
    std::vector<NpDist> rnd((size_t)std::max(RL, 1));
    for (int r = 0; r < RL; r++) {
        rdist[r] = (s->rl_dist && !s->rl_user[r]) ? s->rl_dist[r] : 1;
        if (rdist[r] == 2) rnd[r] = np_dist_binomial(s->rl_n[r], s->rl_dp[r]);
        if (rdist[r] == 3) rnd[r] = np_dist_integers(s->rl_n[r], s->rl_high[r] - 1);
        if (rdist[r] == 4) rnd[r] = np_dist_geometric(s->rl_dp[r]);
        any_int = any_int || rdist[r] == 3;
        any_npd = any_npd || rdist[r] > 1;
    }
    // numpy's buffered 32-bit half of the bit generator (integers markets only)
    const int64_t o_U32 = any_int ? lay.add("u32buf", 8, 1, h->Npad) : -1;
    Blob tb;
    int64_t t_I0 = tb.put(s->I0, J), t_h = tb.put(s->h, J), t_C = tb.put(s->C, J),
            t_o = tb.put(s->o, J), t_v = tb.put(s->v, J);
    int64_t t_if = tb.put(s->is_factory, J), t_ir = tb.put(s->is_retail, J);
    int64_t t_sup = tb.put(s->sup, E), t_pur = tb.put(s->pur, E), t_sf = tb.put(s->sup_is_factory, E),
            t_L = tb.put(s->L, E), t_lp = tb.put(s->lp, E), t_lg = tb.put(s->lg, E);
    std::vector<int32_t> roff((size_t)std::max(E, 1), 0);
    for (int k = 0, off = 0; k < E; k++) {
        roff[k] = off;
        off += s->L[k];
    }
    int64_t t_ro = tb.put(roff.data(), roff.size());
    std::vector<int32_t> woff((size_t)std::max(E, 1), 0);  // obs offset of each link's order window
    for (int k = 0, off = RL + J; k < E; k++) {
        woff[k] = off;
        off += s->L[k];
    }
    int64_t t_wo = tb.put(woff.data(), woff.size());
    int64_t t_rn = tb.put(s->rl_node, RL), t_ru = tb.put(s->rl_user, RL), t_rp = tb.put(s->rl_p, RL),
            t_rb = tb.put(s->rl_b, RL);
    std::vector<PtrsConst> pcs((size_t)std::max(RL, 1));
    std::vector<double> rhs;
    for (int r = 0; r < RL; r++) {
        pcs[r] = ptrs_const(s->rl_user[r] ? 0.0 : s->rl_lam[r]);
        rhs_table(pcs[r], rhs);
    }
    int64_t t_pc = tb.put(pcs.data(), pcs.size());
    int64_t t_rhs = tb.put(rhs.data(), rhs.size());
    int64_t t_rd = tb.put(rdist.data(), rdist.size()), t_rnd = tb.put(rnd.data(), rnd.size());
    std::vector<double> ud((size_t)std::max(RL, 1) * s->num_periods, 0.0);
    if (s->user_D) std::memcpy(ud.data(), s->user_D, sizeof(double) * RL * s->num_periods);
    int64_t t_ud = tb.put(ud.data(), ud.size());
    int64_t t_sp = tb.put(s->succ_ptr, J + 1), t_sk = tb.put(s->succ_kind, nsucc),
            t_sx = tb.put(s->succ_idx, nsucc), t_pp = tb.put(s->pred_ptr, J + 1),
            t_px = tb.put(s->pred_idx, npred);
    std::vector<double> ap((size_t)s->num_periods);
    for (int t = 0; t < s->num_periods; t++) ap[t] = std::pow(s->alpha, (double)t);
    int64_t t_ap = tb.put(ap.data(), ap.size());
    int rc = alloc_arena(h, lay);
    if (rc == INVSIM_OK) rc = upload_tables(h, tb.b);
    if (rc == INVSIM_OK) {
        bind_common(h, o_rng, o_per, o_st, ar);
        NetParams &p = h->net;
        p.J = J;
        p.E = E;
        p.RL = RL;
        p.sumL = sumL;
        if (net_lds_bytes(p) > 160 * 1024) rc = fail(h, INVSIM_ERANGE, "topology too large for the LDS scratch");
    }
    if (rc == INVSIM_OK) {
        NetParams &p = h->net;
        p.cm = h->cm;
        p.J = J;
        p.E = E;
        p.RL = RL;
        p.T = s->num_periods;
        p.backlog = s->backlog != 0;
        p.sumL = sumL;
        p.I0 = tab<double>(h, t_I0);
        p.h = tab<double>(h, t_h);
        p.C = tab<double>(h, t_C);
        p.o = tab<double>(h, t_o);
        p.v = tab<double>(h, t_v);
        p.is_factory = tab<int32_t>(h, t_if);
        p.is_retail = tab<int32_t>(h, t_ir);
        p.sup = tab<int32_t>(h, t_sup);
        p.pur = tab<int32_t>(h, t_pur);
        p.sup_is_factory = tab<int32_t>(h, t_sf);
        p.L = tab<int32_t>(h, t_L);
        p.ring_off = tab<int32_t>(h, t_ro);
        p.lp = tab<double>(h, t_lp);
        p.lg = tab<double>(h, t_lg);
        p.rl_node = tab<int32_t>(h, t_rn);
        p.rl_user = tab<int32_t>(h, t_ru);
        p.rl_p = tab<double>(h, t_rp);
        p.rl_b = tab<double>(h, t_rb);
        p.rl_pc = tab<PtrsConst>(h, t_pc);
        p.rl_dist = any_npd ? tab<int32_t>(h, t_rd) : nullptr;
        p.rl_nd = tab<NpDist>(h, t_rnd);
        if (o_U32 >= 0) h->cm.u32buf = at<uint64_t>(h, o_U32);
        p.cm = h->cm;
        p.rhs = rhs.empty() ? nullptr : tab<double>(h, t_rhs);
        p.win_off = tab<int32_t>(h, t_wo);
        p.user_D = tab<double>(h, t_ud);
        p.succ_ptr = tab<int32_t>(h, t_sp);
        p.succ_kind = tab<int32_t>(h, t_sk);
        p.succ_idx = tab<int32_t>(h, t_sx);
        p.pred_ptr = tab<int32_t>(h, t_pp);
        p.pred_idx = tab<int32_t>(h, t_px);
        p.alpha_pow = tab<double>(h, t_ap);
        p.X = at<double>(h, o_X);
        p.U = at<double>(h, o_U);
        p.Y = at<double>(h, o_Y);
        p.Rring = at<double>(h, o_R);
        rc = init_period(h, s->num_periods);
        // the reference's own graphs run the compile-time specialised kernel
        // (INVSIM_NET_GENERIC=1 forces the generic one, for cross-checks)
        h->net_spec = h->cm.kn.net_generic ? NET_SPEC_NONE : net_spec_match(*s);
        p.ahead = nullptr;
        if (rc == INVSIM_OK && h->net_spec != NET_SPEC_NONE) {   // lookahead cache: 2 slots x (2 + RL) rows
            hipError_t e = hipMalloc(&h->scratch, (size_t)(2 * (2 + p.RL) * h->Npad * sizeof(uint64_t)));
            if (e != hipSuccess) rc = fail(h, INVSIM_ENOMEM, "hipMalloc(lookahead cache)");
            else p.ahead = static_cast<uint64_t *>(h->scratch);
        }
    }
    return finish_create(h, out, rc);
}

// ------------------------------------------------------------------ common entry points
int invsim_dims(const invsim_handle *h, int32_t *obs_dim, int32_t *action_dim, int32_t *demand_dim,
                int32_t *family) {
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (obs_dim) *obs_dim = h->obs_dim;
    if (action_dim) *action_dim = h->act_dim;
    if (demand_dim) *demand_dim = h->demand_dim;
    if (family) *family = h->family;
    return INVSIM_OK;
}

static void sync_common(invsim_handle *h) {
    h->nv.cm = h->cm;
    h->im.cm = h->cm;
    h->net.cm = h->cm;
}

// the fast stream's counter into the kernel parameters (after set_state: from
// the blob first, which is the one synchronising read of that stream)
static int ph_counter_sync(invsim_handle *h, hipStream_t s) {
    if (h->ph_from_blob) {
        hipError_t e = hipMemcpyAsync(&h->ph_step, h->arena + h->o_phstep, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(h, e, "philox_step read");
        h->ph_from_blob = false;
    }
    h->cm.ph_step = h->ph_step;
    sync_common(h);
    return INVSIM_OK;
}


int invsim_set_autoreset(invsim_handle *h, int32_t mode) {
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (int rc = refuse_in_capture(h, "set_autoreset")) return rc;
    if (!valid_autoreset(mode)) return fail(h, INVSIM_EINVAL, "bad autoreset mode");
    h->cm.autoreset = mode;
    sync_common(h);
    return INVSIM_OK;
}

static int info_record_dim(const invsim_handle *h) {
    if (h->family == INVSIM_INVMGMT) return 2 * (h->im_m1 + 1) + 5;
    if (h->family == INVSIM_NETINVMGMT) return 2 * h->net.RL + 2 * h->net.J + 2 * h->net.E;
    if (h->family == INVSIM_NEWSVENDOR) return 5;
    return 0;
}

int invsim_info_record_dim(const invsim_handle *h, int32_t *dim) {
    if (!h || !dim) return fail(nullptr, INVSIM_EINVAL, "null argument");
    *dim = info_record_dim(h);
    return INVSIM_OK;
}

int invsim_set_info_record(invsim_handle *h, void *record) {
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (int rc = refuse_in_capture(h, "set_info_record")) return rc;
    if (record && info_record_dim(h) == 0) return fail(h, INVSIM_EINVAL, "this env family has no step record");
    h->cm.info_rec = record;
    sync_common(h);
    return INVSIM_OK;
}

int invsim_set_info_demand(invsim_handle *h, int64_t *demand) {
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (int rc = refuse_in_capture(h, "set_info_demand")) return rc;
    h->cm.info_demand = demand;
    sync_common(h);
    return INVSIM_OK;
}

// bring cm.rng up to date from the demand lookahead cache (the cache stays valid)
static int commit_rng(invsim_handle *h, hipStream_t s) {
    // a fast-stream cache holds demands only (set_demand_stream drops the other kind)
    if (!h->la_valid || h->demand_stream == INVSIM_DEMAND_PHILOX) return INVSIM_OK;
    hipError_t e = hipSuccess;
    if (h->family == INVSIM_INVMGMT) e = im_commit_launch(h->im, h->la_slot, s);
    else if (h->family == INVSIM_NEWSVENDOR) e = nv_commit_launch(h->nv, h->la_slot, s);
    else if (h->family == INVSIM_NETINVMGMT) e = net_commit_launch(h->net, h->la_slot, s);
    return e == hipSuccess ? INVSIM_OK : hip_fail(h, e, "rng commit");
}

// An unmasked seed restarts the fast stream's launch-step counter, so the same
// seeds give the same demands again (gymnasium's reset(seed=s) contract); a
// masked one keeps it, since the other envs' streams continue.
static void ph_counter_restart(invsim_handle *h) {
    h->ph_step = 0;
    h->ph_from_blob = false;
    h->cm.ph_step = 0;
    sync_common(h);
}

int invsim_seed_range(invsim_handle *h, uint64_t base_lo, uint64_t base_hi, int64_t first,
                      const uint8_t *mask, void *stream) {
    TraceRange tr_("invsim_seed_range");
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (first < 0) return fail(h, INVSIM_EINVAL, "first_index must be >= 0");
    if (int rc = capture_check(h, (hipStream_t)stream)) return rc;
    DeviceGuard g(h->device);
    int rc = commit_rng(h, (hipStream_t)stream);   // a masked seed keeps the other streams
    if (rc != INVSIM_OK) return rc;
    h->la_valid = false;   // the lookahead cache follows the old streams
    if (!mask) ph_counter_restart(h);
    hipError_t e = seed_range_launch(h->cm, base_lo, base_hi, first, mask, (hipStream_t)stream);
    return e == hipSuccess ? INVSIM_OK : hip_fail(h, e, "seed_range launch");
}

int invsim_seed_words(invsim_handle *h, const uint32_t *words, const int32_t *nwords,
                      const uint8_t *mask, void *stream) {
    TraceRange tr_("invsim_seed_words");
    if (!h || (!words && h->N) || (!nwords && h->N)) return fail(h, INVSIM_EINVAL, "null argument");
    if (int rc = capture_check(h, (hipStream_t)stream)) return rc;
    DeviceGuard g(h->device);
    int rc = commit_rng(h, (hipStream_t)stream);
    if (rc != INVSIM_OK) return rc;
    h->la_valid = false;
    if (!mask) ph_counter_restart(h);
    hipError_t e = seed_words_launch(h->cm, words, nwords, mask, (hipStream_t)stream);
    return e == hipSuccess ? INVSIM_OK : hip_fail(h, e, "seed_words launch");
}

// materialise the lock-step period into the per-env row before it stops being uniform
static int materialize_period(invsim_handle *h, hipStream_t s) {
    if (!h->t_known) return INVSIM_OK;
    hipError_t e = period_fill_launch(h->cm, h->t_cur, s);
    return e == hipSuccess ? INVSIM_OK : hip_fail(h, e, "period fill");
}

int invsim_reset(invsim_handle *h, const uint8_t *mask, void *obs, void *stream) {
    TraceRange tr_("invsim_reset");
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (int rc = capture_check(h, (hipStream_t)stream)) return rc;
    if (h->capturing && h->demand_stream == INVSIM_DEMAND_PHILOX)
        return fail(h, INVSIM_EINVAL, "graph capture needs the numpy demand stream");
    DeviceGuard g(h->device);
    hipStream_t s = (hipStream_t)stream;
    if (mask) {
        int rc = materialize_period(h, s);
        if (rc != INVSIM_OK) return rc;
    }
    if (h->family == INVSIM_NEWSVENDOR) {   // its reset draws from cm.rng (or the fast stream)
        int rc = commit_rng(h, s);
        if (rc != INVSIM_OK) return rc;
        h->la_valid = false;
        if (h->demand_stream == INVSIM_DEMAND_PHILOX) {
            rc = ph_counter_sync(h, s);
            if (rc != INVSIM_OK) return rc;
            h->ph_step += 1;                  // the reset's uniforms own a counter value
        }
    }
    hipError_t e = hipSuccess;
    switch (h->family) {
        case INVSIM_NEWSVENDOR: e = nv_reset_launch(h->nv, mask, (float *)obs, s); break;
        case INVSIM_INVMGMT: e = im_reset_launch(h->im, h->im_m1, h->im_backlog, mask, (int64_t *)obs, s); break;
        case INVSIM_NETINVMGMT: e = net_reset_launch(h->net, mask, (float *)obs, s); break;
        default: return fail(h, INVSIM_EINVAL, "bad handle family");
    }
    if (e != hipSuccess) return hip_fail(h, e, "reset launch");
    if (mask) {
        h->t_known = false;
    } else {
        h->t_known = true;
        h->t_cur = 0;
    }
    return INVSIM_OK;
}

static int run_steps(invsim_handle *h, int K, const void *actions, void *obs, double *reward,
                     uint8_t *terminated, uint8_t *truncated, void *final_obs, hipStream_t s,
                     const PolicyIO *pol = nullptr) {
    if (int rc = capture_check(h, s)) return rc;
    if (h->capturing) {
        if (h->demand_stream == INVSIM_DEMAND_PHILOX)
            return fail(h, INVSIM_EINVAL, "graph capture needs the numpy demand stream: the fast stream's launch-step "
                                          "counter is a launch parameter and would repeat on every replay");
        if (!h->t_known && h->cm.autoreset == AR_DISABLED && !h->past_ok)
            return fail(h, INVSIM_EINVAL, "graph capture of steps with autoreset DISABLED after a masked reset: "
                                          "the horizon check reads the device status word (a host synchronisation)");
        h->cap_steps += K;
    }
    int t_u = -1;
    if (h->t_known) {
        t_u = h->t_cur;
        // DISABLED autoreset: refuse to step InvMgmt/NetInvMgmt past the horizon
        // (the reference raises IndexError, inventory_management.py:267)
        int t = h->t_cur;
        for (int k = 0; k < K; k++) {
            if (t >= h->horizon && h->cm.autoreset == AR_DISABLED && !h->past_ok)
                return fail(h, INVSIM_ERANGE, "step past the episode horizon with autoreset disabled; reset first");
            t = next_period(t, h->horizon, h->cm.autoreset, h->past_ok);
        }
    }
    if (h->demand_stream == INVSIM_DEMAND_PHILOX) {
        int rc = ph_counter_sync(h, s);
        if (rc != INVSIM_OK) return rc;
    }
    // episode sink: a kernel that does not fold in-kernel leaves it to the
    // group fold of its output rows below (the same arithmetic, kernels.hpp EpSink)
    if (h->cm.ep_ret && h->N && !reward)
        return fail(h, INVSIM_EINVAL, "the episode sink folds the reward outputs: pass reward / terminated / truncated");
    bool sunk = false;
    hipError_t e = hipSuccess;
    switch (h->family) {
        case INVSIM_NEWSVENDOR: {
            StepIO<float, float> io{K, (const float *)actions, (float *)obs, reward, terminated, truncated, (float *)final_obs};
            e = nv_run_launch(h->nv, t_u, pol, io, h->la_valid, h->la_slot, s);
            break;
        }
        case INVSIM_INVMGMT: {
            StepIO<int64_t, int64_t> io{K, (const int64_t *)actions, (int64_t *)obs, reward, terminated, truncated,
                                        (int64_t *)final_obs};
            e = im_run_launch(h->im, h->im_m1, h->im_backlog, t_u, pol, io, h->la_valid, h->la_slot, sunk, s);
            break;
        }
        case INVSIM_NETINVMGMT: {
            StepIO<float, float> io{K, (const float *)actions, (float *)obs, reward, terminated, truncated, (float *)final_obs};
            e = h->net_spec ? net_spec_launch(h->net_spec, h->net, t_u, pol, io, h->la_valid, h->la_slot, s)
                            : net_run_launch(h->net, t_u, pol, io, s);
            break;
        }
        default: return fail(h, INVSIM_EINVAL, "bad handle family");
    }
    if (e != hipSuccess) {
        h->la_valid = false;
        return hip_fail(h, e, "step launch");
    }
    if (h->cm.ep_ret && !sunk) {
        if (!reward) return fail(h, INVSIM_EINVAL, "the episode sink needs this launch's reward outputs");
        e = episode_fold_groups_launch(reward, terminated, truncated, K, h->N, h->cm.ep_ret, h->cm.ep_part, s);
        if (e != hipSuccess) return hip_fail(h, e, "episode sink fold");
    }
    if (h->demand_stream == INVSIM_DEMAND_PHILOX) h->ph_step += (uint64_t)K;   // one counter value per launch step
    if (h->t_known) {
        for (int k = 0; k < K; k++) h->t_cur = next_period(h->t_cur, h->horizon, h->cm.autoreset, h->past_ok);
    } else if (h->cm.autoreset == AR_DISABLED && !h->past_ok) {
        // per-env periods (after a masked reset): the kernels skip an env stepped
        // past its horizon and flag it; surface that now, as the reference's
        // IndexError (inventory_management.py:267), at the cost of one sync
        uint32_t flags = 0;
        e = hipMemcpyAsync(&flags, h->cm.status, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(h, e, "status read");
        if (flags & 1u) {
            e = hipMemsetAsync(h->cm.status, 0, sizeof(uint32_t), s);
            if (e != hipSuccess) return hip_fail(h, e, "status clear");
            return fail(h, INVSIM_ERANGE,
                        "an env was stepped past its episode horizon with autoreset disabled (that env's step was "
                        "not applied; its outputs are undefined); reset it first");
        }
    }
    return INVSIM_OK;
}

int invsim_step(invsim_handle *h, const void *actions, void *obs, double *reward, uint8_t *terminated,
                uint8_t *truncated, void *final_obs, void *stream) {
    TraceRange tr_("invsim_step");
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (h->N && (!actions || !obs || !reward || !terminated || !truncated))
        return fail(h, INVSIM_EINVAL, "null output/input buffer");
    DeviceGuard g(h->device);
    return run_steps(h, 1, actions, obs, reward, terminated, truncated,
                     h->cm.autoreset == AR_SAME_STEP ? final_obs : nullptr, (hipStream_t)stream);
}

int invsim_rollout(invsim_handle *h, int32_t K, const void *actions, void *obs, double *reward,
                   uint8_t *terminated, uint8_t *truncated, void *stream) {
    TraceRange tr_("invsim_rollout");
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (K < 0) return fail(h, INVSIM_EINVAL, "K must be >= 0");
    if (K == 0) return INVSIM_OK;
    if (h->N && (!actions || !obs || !reward || !terminated || !truncated))
        return fail(h, INVSIM_EINVAL, "null output/input buffer");
    if (h->cm.autoreset == AR_SAME_STEP)
        return fail(h, INVSIM_EINVAL, "rollout does not return final_obs: use NEXT_STEP or DISABLED autoreset");
    DeviceGuard g(h->device);
    return run_steps(h, K, actions, obs, reward, terminated, truncated, nullptr, (hipStream_t)stream);
}

static int metrics_dim(const invsim_handle *h) {
    switch (h->family) {
        case INVSIM_NEWSVENDOR: return 2;
        case INVSIM_INVMGMT: return 6;
        case INVSIM_NETINVMGMT: return 5 + h->net.J;
        default: return 0;
    }
}

int invsim_metrics_dim(const invsim_handle *h, int32_t *dim) {
    if (!h || !dim) return fail(nullptr, INVSIM_EINVAL, "null argument");
    *dim = metrics_dim(h);
    return INVSIM_OK;
}

int invsim_rollout_policy(invsim_handle *h, int32_t K, const invsim_policy *policy, void *obs, double *reward,
                          uint8_t *terminated, uint8_t *truncated, void *actions, double *metrics, void *stream) {
    TraceRange tr_("invsim_rollout_policy");
    if (!h || !policy) return fail(h, INVSIM_EINVAL, "null argument");
    if (K < 0) return fail(h, INVSIM_EINVAL, "K must be >= 0");
    if (K == 0) return INVSIM_OK;
    if (h->cm.autoreset == AR_SAME_STEP)
        return fail(h, INVSIM_EINVAL, "policy rollouts do not return final_obs: use NEXT_STEP or DISABLED autoreset");
    if ((reward == nullptr) != (terminated == nullptr) || (reward == nullptr) != (truncated == nullptr))
        return fail(h, INVSIM_EINVAL, "reward, terminated and truncated are given together or not at all");
    PolicyIO p{};
    p.kind = policy->kind;
    p.variant = policy->variant;
    p.sf = policy->safety_factor;
    p.mu = policy->mu;
    p.act_out = actions;
    p.metrics = metrics;
    p.mdim = metrics_dim(h);
    switch (policy->kind) {
        case INVSIM_POLICY_CONSTANT:
            if (!policy->constant) return fail(h, INVSIM_EINVAL, "CONSTANT policy needs its action vector");
            if (h->act_dim > POL_MAX_A) return fail(h, INVSIM_ERANGE, "action_dim too large for a CONSTANT policy");
            for (int a = 0; a < h->act_dim; a++) {
                if (h->family == INVSIM_INVMGMT) p.ci[a] = ((const int64_t *)policy->constant)[a];
                else p.cf[a] = ((const float *)policy->constant)[a];
            }
            break;
        case INVSIM_POLICY_BASE_STOCK:
            if (h->family != INVSIM_INVMGMT) return fail(h, INVSIM_EINVAL, "BASE_STOCK is an InvMgmt policy");
            break;
        case INVSIM_POLICY_ORDER_UP_TO:
            if (h->family != INVSIM_NEWSVENDOR) return fail(h, INVSIM_EINVAL, "ORDER_UP_TO is a Newsvendor policy");
            break;
        case INVSIM_POLICY_CLASSIC_NV:
        case INVSIM_POLICY_SS: {
            if (h->family != INVSIM_NEWSVENDOR)
                return fail(h, INVSIM_EINVAL, "CLASSIC_NV / SS are Newsvendor policies");
            if (policy->kind == INVSIM_POLICY_CLASSIC_NV && (policy->variant < 0 || policy->variant > 1))
                return fail(h, INVSIM_EINVAL, "CLASSIC_NV variant: 0 'k_vs_h' or 1 'profit_margin'");
            // the device ppf walks the Poisson CDF: bounded work per env
            const double sf = policy->kind == INVSIM_POLICY_CLASSIC_NV ? policy->safety_factor : 1.0;
            const double lam = (double)(float)h->nv.mu_max * (h->nv.L + 1) * (sf > 1 ? sf : 1.0);
            if (!(lam <= 1e6))
                return fail(h, INVSIM_ERANGE, "critical-ratio policies need mu_max * (lead_time + 1) * safety_factor <= 1e6");
            break;
        }
        default: return fail(h, INVSIM_EINVAL, "unknown policy kind");
    }
    DeviceGuard g(h->device);
    return run_steps(h, K, nullptr, obs, reward, terminated, truncated, nullptr, (hipStream_t)stream, &p);
}

int invsim_episode_fold(const double *reward, const uint8_t *terminated, const uint8_t *truncated, int32_t K,
                        int64_t n_envs, double *ret, double *acc, void *stream) {
    TraceRange tr_("invsim_episode_fold");
    if (!reward || !ret || !acc || K < 0 || n_envs < 0)
        return fail(nullptr, INVSIM_EINVAL, "episode_fold: null buffer or negative size");
    hipError_t e = episode_fold_launch(reward, terminated, truncated, K, n_envs, ret, acc, (hipStream_t)stream);
    return e == hipSuccess ? INVSIM_OK : hip_fail(nullptr, e, "episode_fold launch");
}

int invsim_episode_fold_groups(const double *reward, const uint8_t *terminated, const uint8_t *truncated,
                               int32_t K, int64_t n_envs, double *ret, double *part, void *stream) {
    TraceRange tr_("invsim_episode_fold_groups");
    if ((!reward && K > 0 && n_envs > 0) || !ret || !part || K < 0 || n_envs < 0)
        return fail(nullptr, INVSIM_EINVAL, "episode_fold_groups: null buffer or negative size");
    hipError_t e = episode_fold_groups_launch(reward, terminated, truncated, K, n_envs, ret, part, (hipStream_t)stream);
    return e == hipSuccess ? INVSIM_OK : hip_fail(nullptr, e, "episode_fold_groups launch");
}

int invsim_set_episode_sink(invsim_handle *h, double *ret, double *part) {
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (int rc = refuse_in_capture(h, "set_episode_sink")) return rc;
    if ((ret == nullptr) != (part == nullptr)) return fail(h, INVSIM_EINVAL, "episode sink: ret and part together");
    h->cm.ep_ret = ret;
    h->cm.ep_part = part;
    sync_common(h);
    return INVSIM_OK;
}

int invsim_debug_ptrs_stats(uint64_t *out, int32_t clear) {
    if (!out) return fail(nullptr, INVSIM_EINVAL, "null argument");
#ifdef INVSIM_PTRS_STATS
    hipError_t (*tus[6])(unsigned long long *, bool) = {ptrs_stats_nv, ptrs_stats_nv_ph, ptrs_stats_im,
                                                        ptrs_stats_im_ph, ptrs_stats_netspec, ptrs_stats_net};
    out[0] = out[1] = out[3] = out[4] = 0;
    out[2] = 0x7ff0000000000000ull;
    for (auto f : tus) {
        unsigned long long v[5];
        hipError_t e = hipDeviceSynchronize();
        if (e == hipSuccess) e = f(v, clear != 0);
        if (e != hipSuccess) return hip_fail(nullptr, e, "ptrs stats");
        out[0] += v[0];
        out[1] += v[1];
        out[3] += v[3];
        out[4] += v[4];
        out[2] = std::min<uint64_t>(out[2], v[2]);
    }
    return INVSIM_OK;
#else
    (void)clear;
    return fail(nullptr, INVSIM_EINVAL, "not a PTRS-statistics build (make -C csrc ptrs_stats)");
#endif
}

int invsim_set_demand_stream(invsim_handle *h, int32_t mode) {
    TraceRange tr_("invsim_set_demand_stream");
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (int rc = refuse_in_capture(h, "set_demand_stream")) return rc;
    if (mode != INVSIM_DEMAND_NUMPY && mode != INVSIM_DEMAND_PHILOX)
        return fail(h, INVSIM_EINVAL, "demand stream must be INVSIM_DEMAND_NUMPY or INVSIM_DEMAND_PHILOX");
    if (mode == h->demand_stream) return INVSIM_OK;
    DeviceGuard g(h->device);
    // steps may still be queued on a caller's non-blocking stream, which the
    // legacy stream does not wait for: drain the device before the commit reads
    // the lookahead slot those steps write
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return hip_fail(h, e, "demand stream switch");
    int rc = commit_rng(h, nullptr);   // the parity stream's lookahead cache ends (legacy stream)
    if (rc != INVSIM_OK) return rc;
    e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) return hip_fail(h, e, "demand stream switch");
    h->la_valid = false;
    h->demand_stream = mode;
    h->cm.philox = mode == INVSIM_DEMAND_PHILOX ? 1 : 0;
    sync_common(h);
    return INVSIM_OK;
}

int invsim_demand_stream(const invsim_handle *h, int32_t *mode) {
    if (!h || !mode) return fail(nullptr, INVSIM_EINVAL, "null argument");
    *mode = h->demand_stream;
    return INVSIM_OK;
}

int invsim_kernel_variant(const invsim_handle *h, int32_t *variant) {
    if (!h || !variant) return fail(nullptr, INVSIM_EINVAL, "null argument");
    *variant = h->family == INVSIM_NETINVMGMT ? h->net_spec : 0;
    return INVSIM_OK;
}

int invsim_status(invsim_handle *h, uint32_t *flags, int32_t clear) {
    if (!h || !flags) return fail(h, INVSIM_EINVAL, "null argument");
    if (int rc = refuse_in_capture(h, "status")) return rc;
    DeviceGuard g(h->device);
    hipError_t e = hipMemcpy(flags, h->cm.status, sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(h, e, "status read");
    if (clear && *flags) {
        e = hipMemset(h->cm.status, 0, sizeof(uint32_t));
        if (e != hipSuccess) return hip_fail(h, e, "status clear");
    }
    return INVSIM_OK;
}

int invsim_state_bytes(const invsim_handle *h, int64_t *bytes) {
    if (!h || !bytes) return fail(nullptr, INVSIM_EINVAL, "null argument");
    *bytes = h->arena_bytes;
    return INVSIM_OK;
}

int invsim_state_field(const invsim_handle *h, int32_t idx, char name[32], int64_t *offset,
                       int32_t *elem_bytes, int32_t *rows, int64_t *row_stride) {
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (idx < 0 || idx >= (int32_t)h->fields.size()) return INVSIM_ERANGE;
    const Field &f = h->fields[idx];
    if (name) {
        std::memset(name, 0, 32);
        std::strncpy(name, f.name.c_str(), 31);
    }
    if (offset) *offset = f.offset;
    if (elem_bytes) *elem_bytes = f.elem;
    if (rows) *rows = f.rows;
    // > 0: [rows][row_stride]; < 0: record layout [-row_stride][rows]; 0: other layout
    if (row_stride) *row_stride = (f.name == "status" || f.name == "philox_step") ? 1 : f.kind == 1 ? -h->Npad : f.kind == 2 ? 0 : h->Npad;
    return INVSIM_OK;
}

int invsim_get_state(invsim_handle *h, void *dst, void *stream) {
    TraceRange tr_("invsim_get_state");
    if (!h || !dst) return fail(h, INVSIM_EINVAL, "null argument");
    if (int rc = refuse_in_capture(h, "get_state")) return rc;
    DeviceGuard g(h->device);
    int rc = materialize_period(h, (hipStream_t)stream);  // the blob carries per-env periods
    if (rc == INVSIM_OK) rc = commit_rng(h, (hipStream_t)stream);   // and the committed PCG64 states
    if (rc != INVSIM_OK) return rc;
    if (!h->ph_from_blob) {                                // and the fast stream's counter
        hipError_t e0 = hipMemcpyAsync(h->arena + h->o_phstep, &h->ph_step, sizeof(uint64_t),
                                       hipMemcpyHostToDevice, (hipStream_t)stream);
        if (e0 == hipSuccess) e0 = hipStreamSynchronize((hipStream_t)stream);   // the host word may change next
        if (e0 != hipSuccess) return hip_fail(h, e0, "philox_step write");
    }
    hipError_t e = hipMemcpyAsync(dst, h->arena, (size_t)h->arena_bytes, hipMemcpyDeviceToDevice,
                                  (hipStream_t)stream);
    return e == hipSuccess ? INVSIM_OK : hip_fail(h, e, "get_state");
}

int invsim_set_state(invsim_handle *h, const void *src, void *stream) {
    TraceRange tr_("invsim_set_state");
    if (!h || !src) return fail(h, INVSIM_EINVAL, "null argument");
    if (int rc = refuse_in_capture(h, "set_state")) return rc;
    DeviceGuard g(h->device);
    hipError_t e = hipMemcpyAsync(h->arena, src, (size_t)h->arena_bytes, hipMemcpyDeviceToDevice,
                                  (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(h, e, "set_state");
    h->t_known = false;  // periods now come from the blob
    h->la_valid = false;
    h->ph_from_blob = true;   // and the fast stream's counter (read when next needed)
    return INVSIM_OK;
}

// ------------------------------------------------------------------ graph capture
int invsim_capture_begin(invsim_handle *h) {
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (h->capturing) return fail(h, INVSIM_EINVAL, "capture_begin: this handle is already capturing");
    if (h->demand_stream == INVSIM_DEMAND_PHILOX)
        return fail(h, INVSIM_EINVAL, "graph capture needs the numpy demand stream: the fast stream's launch-step "
                                      "counter is a launch parameter and would repeat on every replay");
    h->capturing = true;
    h->cap_t_known = h->t_known;
    h->cap_t_cur = h->t_cur;
    h->cap_la_valid = h->la_valid;
    h->cap_la_slot = h->la_slot;
    h->cap_steps = 0;
    return INVSIM_OK;
}

int invsim_capture_end(invsim_handle *h, int64_t *steps) {
    if (!h) return fail(nullptr, INVSIM_EINVAL, "null handle");
    if (!h->capturing) return fail(h, INVSIM_EINVAL, "capture_end without capture_begin");
    if (steps) *steps = h->cap_steps;
    const bool closed = h->t_known == h->cap_t_known && (!h->t_known || h->t_cur == h->cap_t_cur) &&
                        h->la_valid == h->cap_la_valid && (!h->la_valid || h->la_slot == h->cap_la_slot);
    const int32_t t_end = h->t_known ? h->t_cur : -1;
    const bool la_end = h->la_valid;
    // nothing ran: the device is still where capture_begin found it
    h->capturing = false;
    h->t_known = h->cap_t_known;
    h->t_cur = h->cap_t_cur;
    h->la_valid = h->cap_la_valid;
    h->la_slot = h->cap_la_slot;
    if (closed) return INVSIM_OK;
    std::string msg = "the captured calls (" + std::to_string(h->cap_steps) + " env steps) move the handle from period " +
                      std::to_string(h->t_known ? h->t_cur : -1) + " to " + std::to_string(t_end);
    if (la_end != h->la_valid) msg += " and change the demand lookahead state";
    msg += ": a replay would not start where the graph was recorded; capture a whole number of episode cycles (" +
           std::to_string(h->horizon + (h->cm.autoreset == AR_NEXT_STEP ? 1 : 0)) +
           " steps) from a handle that has already stepped once";
    return fail(h, INVSIM_ERANGE, msg);
}

int invsim_position(const invsim_handle *h, int64_t *pos) {
    if (!h || !pos) return fail(nullptr, INVSIM_EINVAL, "null argument");
    const uint64_t t = h->t_known ? (uint32_t)h->t_cur : 0xFFFFFFFFu;
    const uint64_t la = h->la_valid ? 2u + (uint64_t)(h->la_slot & 1) : 0u;
    *pos = (int64_t)(t | (la << 32) | ((uint64_t)(h->demand_stream & 1) << 34));
    return INVSIM_OK;
}

}  // extern "C"
