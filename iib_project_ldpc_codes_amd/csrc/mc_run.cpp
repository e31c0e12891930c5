// ldpc_mc_run / ldpc_mc_run_csr: a whole Monte-Carlo run over several devices of
// ONE process.
//
// Reference: the trial loop of run_simulation / run_simulation_fixed_ldpc
// (parallel_simulator.py:198-244, :354-379; expurgated :200-256), which the
// reference parallelises by launching independent processes
// (parallel_simulator.py:403-445) and merging their CSV files afterwards
// (tools/combine_data.py:64-95).
//
// Here: device slot r of round R decodes trials [(R*ndev + r)*batch, +batch) with
// the fused channel + decode + counter kernels (ldpc_mc_batch_dev /
// ldpc_mc_ensemble_batch_dev) on its own stream, launched from its own host thread;
// per round ONE ncclAllReduce
// (sum, int64) of [counter deltas | per-slot frame errors] over the devices
// (RCCL, ncclCommInitAll; over xGMI on an MI355X node).  The stop rule is the
// reference's `while frame_errors < stop and trials < num_tests` in global trial
// order: the last round's batches are clamped to num_tests, and in the round that
// crosses `stop` the slots before the crossing keep their batch, the crossing slot
// re-runs its batch (Philox streams are keyed by trial index) with the in-batch
// cut at its share, and later slots drop theirs.  Same trial partition and result
// as montecarlo.MonteCarlo over W ranks.  The accounting is mc_plan.hpp's, shared with the
// host-only ldpc_debug_mc_plan (tested on the CPU for ndev = 1..8).
//
// RCCL is loaded at first use with dlopen(RTLD_LOCAL), so a process that also
// holds torch's own RCCL copy keeps the two apart.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ldpc_internal.hpp"
#include "ldpc_mi355x.h"
#include "mc_plan.hpp"

using namespace ldpc;

namespace {

struct Rccl {
    void *h = nullptr;
    ncclResult_t (*commInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*allReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    const char *(*errorString)(ncclResult_t) = nullptr;
};

std::mutex g_run_mu;  // one multi-device run at a time (the comms and streams below)
Rccl g_rccl;
// Per device list: RCCL communicators and one stream per device, kept for the
// process lifetime (the per-(device, stream) workspaces of capi.cpp are reused).
struct Ctx {
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> streams;
};
std::map<std::vector<int>, Ctx> g_ctx;

int load_rccl() {
    if (g_rccl.h) return LDPC_OK;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        set_error(std::string("ldpc_mc_run: cannot load RCCL (librccl.so.1): ") + dlerror());
        return LDPC_EUNSUP;
    }
    Rccl r;
    r.h = h;
    r.commInitAll = reinterpret_cast<decltype(r.commInitAll)>(dlsym(h, "ncclCommInitAll"));
    r.allReduce = reinterpret_cast<decltype(r.allReduce)>(dlsym(h, "ncclAllReduce"));
    r.groupStart = reinterpret_cast<decltype(r.groupStart)>(dlsym(h, "ncclGroupStart"));
    r.groupEnd = reinterpret_cast<decltype(r.groupEnd)>(dlsym(h, "ncclGroupEnd"));
    r.errorString = reinterpret_cast<decltype(r.errorString)>(dlsym(h, "ncclGetErrorString"));
    if (!r.commInitAll || !r.allReduce || !r.groupStart || !r.groupEnd || !r.errorString) {
        set_error("ldpc_mc_run: RCCL library lacks ncclCommInitAll / ncclAllReduce / ncclGroupStart/End");
        dlclose(h);
        return LDPC_EUNSUP;
    }
    g_rccl = r;
    return LDPC_OK;
}

#define RUN_HIP(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess) {                                                            \
            set_error(std::string("ldpc_mc_run: " #expr ": ") + hipGetErrorString(_e));    \
            return LDPC_EHIP;                                                              \
        }                                                                                  \
    } while (0)

#define RUN_NCCL(expr)                                                                                      \
    do {                                                                                                    \
        ncclResult_t _r = (expr);                                                                           \
        if (_r != ncclSuccess) {                                                                            \
            set_error(std::string("ldpc_mc_run: " #expr ": ") + g_rccl.errorString(_r));                    \
            return LDPC_EHIP;                                                                               \
        }                                                                                                   \
    } while (0)

// Per-device state of one run.
struct Slot {
    int dev = 0;
    hipStream_t stream = nullptr;
    ldpc_graph *g = nullptr;  // fixed code (nullptr: ensemble mode)
    int64_t *d_send = nullptr, *d_recv = nullptr, *d_tmp = nullptr;  // C + ndev int64 each
};

struct Run {
    // graph source: lists, CSR, or ensemble
    const int32_t *v2c = nullptr, *c2v = nullptr;
    const int32_t *cptr = nullptr, *cvar = nullptr, *vptr = nullptr, *vslot = nullptr;
    int n = 0, k = 0, m = 0, dv = 0, dc = 0;
    bool ensemble = false;
    int channel = 0, algo = 0, early_stop = 0, max_iters = 0, expurgation = -1, batch = 0;
    float param = 0.f, alpha = 1.f;
    uint64_t seed = 0;
};

int launch_batch(const Run &r, Slot &s, uint64_t first_cw, int B, int64_t stop, int64_t *d_counters) {
    if (B <= 0) return LDPC_OK;
    if (r.ensemble)
        return ldpc_mc_ensemble_batch_dev(r.n, r.dv, r.dc, r.channel, r.param, r.seed, first_cw, B, r.max_iters,
                                          r.expurgation, stop, d_counters, s.stream);
    return ldpc_mc_batch_dev(s.g, r.channel, r.param, r.seed, first_cw, B, r.max_iters, r.algo, r.alpha,
                             r.early_stop, r.expurgation, stop, d_counters, s.stream);
}

// The devices' side of mc_drive (mc_plan.hpp).  One host thread per device launches that
// device's batch (ldpc_mc_batch_dev takes only its (device, stream) workspace lock, so the
// launches of different devices do not serialise); the per-round all-reduce is one RCCL
// group call over the devices' communicators from the driving thread.
struct DeviceBackend {
    const Run &r;
    std::vector<Slot> &slots;
    const std::vector<ncclComm_t> &comms;
    int C = 0, V = 0, ndev = 0;
    std::vector<int64_t> G, red, tmp;

    DeviceBackend(const Run &r_, std::vector<Slot> &s, const std::vector<ncclComm_t> &c, int C_)
        : r(r_), slots(s), comms(c), C(C_), V(C_ + (int)s.size()), ndev((int)s.size()), G(C_, 0), red(V), tmp(V) {}
    int64_t frames() const { return G[1]; }
    int64_t trials() const { return G[0]; }
    uint64_t first_cw(int64_t R, int i) const { return (uint64_t)(R * ndev + i) * (uint64_t)r.batch; }

    // slot i: zeroed delta, its batch (no cut), its frame errors copied to position C + i
    int launch_slot(int64_t R, int i, int B) {
        Slot &s = slots[i];
        RUN_HIP(hipSetDevice(s.dev));
        RUN_HIP(hipMemsetAsync(s.d_send, 0, sizeof(int64_t) * V, s.stream));
        int rc = launch_batch(r, s, first_cw(R, i), B, 0, s.d_send);
        if (rc) return rc;
        RUN_HIP(hipMemcpyAsync(s.d_send + C + i, s.d_send + 1, sizeof(int64_t), hipMemcpyDeviceToDevice, s.stream));
        return LDPC_OK;
    }
    int round(int64_t R, const std::vector<int> &B, std::vector<int64_t> &f) {
        std::vector<int> rcs(ndev, LDPC_OK);
        std::vector<std::string> errs(ndev);
        if (ndev == 1) {
            rcs[0] = launch_slot(R, 0, B[0]);
        } else {
            std::vector<std::thread> th;
            th.reserve(ndev);
            for (int i = 0; i < ndev; ++i)
                th.emplace_back([&, i]() {
                    rcs[i] = launch_slot(R, i, B[i]);
                    if (rcs[i]) errs[i] = ldpc_last_error();  // the error text is per thread
                });
            for (auto &t : th) t.join();
        }
        for (int i = 0; i < ndev; ++i)
            if (rcs[i]) {
                if (!errs[i].empty()) set_error(errs[i]);
                return rcs[i];
            }
        RUN_NCCL(g_rccl.groupStart());
        for (int i = 0; i < ndev; ++i) {
            Slot &s = slots[i];
            RUN_NCCL(g_rccl.allReduce(s.d_send, s.d_recv, (size_t)V, ncclInt64, ncclSum, comms[i], s.stream));
        }
        RUN_NCCL(g_rccl.groupEnd());
        RUN_HIP(hipSetDevice(slots[0].dev));
        RUN_HIP(hipMemcpyAsync(red.data(), slots[0].d_recv, sizeof(int64_t) * V, hipMemcpyDeviceToHost,
                               slots[0].stream));
        for (auto &s : slots) {
            RUN_HIP(hipSetDevice(s.dev));
            RUN_HIP(hipStreamSynchronize(s.stream));
        }
        for (int i = 0; i < ndev; ++i) f[i] = red[C + i];
        return LDPC_OK;
    }
    int keep_round() {
        for (int j = 0; j < C; ++j) G[j] += red[j];
        return LDPC_OK;
    }
    int keep(int i) {  // slot i's own (un-reduced) delta
        Slot &s = slots[i];
        RUN_HIP(hipSetDevice(s.dev));
        RUN_HIP(hipMemcpy(tmp.data(), s.d_send, sizeof(int64_t) * C, hipMemcpyDeviceToHost));
        for (int j = 0; j < C; ++j) G[j] += tmp[j];
        return LDPC_OK;
    }
    int cut(int64_t R, int i, int B, int64_t quota) {  // the same B trials, cut at the quota
        Slot &s = slots[i];
        RUN_HIP(hipSetDevice(s.dev));
        RUN_HIP(hipMemsetAsync(s.d_tmp, 0, sizeof(int64_t) * V, s.stream));
        int rc = launch_batch(r, s, first_cw(R, i), B, quota, s.d_tmp);
        if (rc) return rc;
        RUN_HIP(hipStreamSynchronize(s.stream));
        RUN_HIP(hipMemcpy(tmp.data(), s.d_tmp, sizeof(int64_t) * C, hipMemcpyDeviceToHost));
        for (int j = 0; j < C; ++j) G[j] += tmp[j];
        return LDPC_OK;
    }
};

int run_impl(const Run &r, int64_t num_tests, int64_t stop, double time_limit_s, const int *devices, int ndev,
             int64_t *counters, int64_t *rounds_out) {
    const int C = LDPC_MC_NCOUNT + r.max_iters + 1;
    const int V = C + ndev;
    int rc = load_rccl();
    if (rc) return rc;
    std::vector<int> devs(devices, devices + ndev);
    int prev_dev = 0;
    RUN_HIP(hipGetDevice(&prev_dev));
    Ctx &ctx = g_ctx[devs];
    if (ctx.comms.empty()) {
        std::vector<ncclComm_t> comms(ndev);
        ncclResult_t nr = g_rccl.commInitAll(comms.data(), ndev, devs.data());
        if (nr != ncclSuccess) {
            g_ctx.erase(devs);
            set_error(std::string("ldpc_mc_run: ncclCommInitAll: ") + g_rccl.errorString(nr));
            return LDPC_EHIP;
        }
        std::vector<hipStream_t> streams(ndev, nullptr);
        for (int i = 0; i < ndev; ++i) {
            RUN_HIP(hipSetDevice(devs[i]));
            RUN_HIP(hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking));
        }
        RUN_HIP(hipSetDevice(prev_dev));
        ctx.comms = comms;
        ctx.streams = streams;
    }
    std::vector<Slot> slots(ndev);
    auto cleanup = [&]() {
        for (auto &s : slots) {
            (void)hipSetDevice(s.dev);
            if (s.stream) (void)hipStreamSynchronize(s.stream);
            if (s.g) ldpc_graph_destroy(s.g);
            if (s.d_send) (void)hipFree(s.d_send);
            if (s.d_recv) (void)hipFree(s.d_recv);
            if (s.d_tmp) (void)hipFree(s.d_tmp);
        }
        (void)hipSetDevice(prev_dev);
    };
    struct Guard {
        std::function<void()> f;
        ~Guard() { f(); }
    } guard{cleanup};

    for (int i = 0; i < ndev; ++i) {
        Slot &s = slots[i];
        s.dev = devs[i];
        RUN_HIP(hipSetDevice(s.dev));
        s.stream = ctx.streams[i];
        RUN_HIP(hipMalloc(&s.d_send, sizeof(int64_t) * V));
        RUN_HIP(hipMalloc(&s.d_recv, sizeof(int64_t) * V));
        RUN_HIP(hipMalloc(&s.d_tmp, sizeof(int64_t) * V));
        if (!r.ensemble) {
            rc = r.v2c ? ldpc_graph_create(r.v2c, r.c2v, r.n, r.k, r.dv, r.dc, &s.g)
                       : ldpc_graph_create_csr(r.cptr, r.cvar, r.vptr, r.vslot, r.n, r.m, &s.g);
            if (rc) return rc;
        }
    }
    McPlan P;
    P.num_tests = num_tests;
    P.stop = stop;
    P.batch = r.batch;
    P.ndev = ndev;
    DeviceBackend be(r, slots, ctx.comms, C);
    int64_t rounds = 0;
    rc = mc_drive(P, be, time_limit_s, rounds);
    if (rc) return rc;
    std::memcpy(counters, be.G.data(), sizeof(int64_t) * C);
    if (rounds_out) *rounds_out = rounds;
    return LDPC_OK;
}

// Host-only stand-in for the devices (ldpc_debug_mc_plan): trial t is a frame error iff
// fe[t] != 0; a batch counts its trials and frame errors, the cut keeps trials up to and
// including the one that reaches the quota (mc_cutoff_kernel's rule).
struct SeqBackend {
    const uint8_t *fe = nullptr;
    int64_t avail = 0;
    int batch = 0, ndev = 0;
    int64_t G[2] = {0, 0};
    std::vector<int64_t> dt, df;  // the round's per-slot deltas
    int64_t frames() const { return G[1]; }
    int64_t trials() const { return G[0]; }
    int count(int64_t first, int B, int64_t quota, int64_t &t, int64_t &f) const {
        t = f = 0;
        if (B > 0 && first + B > avail) {
            set_error("ldpc_debug_mc_plan: the plan reads past the synthetic trial sequence");
            return LDPC_EINVAL;
        }
        for (int j = 0; j < B; ++j) {
            ++t;
            f += fe[first + j] != 0;
            if (quota > 0 && f >= quota) break;
        }
        return LDPC_OK;
    }
    int round(int64_t R, const std::vector<int> &B, std::vector<int64_t> &f) {
        dt.assign(ndev, 0);
        df.assign(ndev, 0);
        for (int i = 0; i < ndev; ++i) {
            int rc = count((R * ndev + i) * (int64_t)batch, B[i], 0, dt[i], df[i]);
            if (rc) return rc;
            f[i] = df[i];
        }
        return LDPC_OK;
    }
    int keep_round() {
        for (int i = 0; i < ndev; ++i) keep(i);
        return LDPC_OK;
    }
    int keep(int i) {
        G[0] += dt[i];
        G[1] += df[i];
        return LDPC_OK;
    }
    int cut(int64_t R, int i, int B, int64_t quota) {
        int64_t t = 0, f = 0;
        int rc = count((R * ndev + i) * (int64_t)batch, B, quota, t, f);
        G[0] += t;
        G[1] += f;
        return rc;
    }
};

int check_common(int channel, int max_iters, int batch, const int *devices, int ndev, int64_t *counters) {
    if (!counters || !devices || ndev <= 0 || max_iters < 0 || batch <= 0) {
        set_error("ldpc_mc_run: need counters, devices[ndev > 0], max_iters >= 0, batch > 0");
        return LDPC_EINVAL;
    }
    if (channel != LDPC_CH_BEC && channel != LDPC_CH_BSC && channel != LDPC_CH_AWGN) {
        set_error("ldpc_mc_run: unknown channel");
        return LDPC_EINVAL;
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        set_error("libldpc_mi355x: no HIP device visible (this library has no CPU path; run on an MI355X)");
        return LDPC_ENODEV;
    }
    for (int i = 0; i < ndev; ++i) {
        if (devices[i] < 0 || devices[i] >= count) {
            set_error("ldpc_mc_run: device ordinal out of range");
            return LDPC_EINVAL;
        }
        for (int j = 0; j < i; ++j)
            if (devices[j] == devices[i]) {
                set_error("ldpc_mc_run: a device is listed twice (RCCL needs one rank per device)");
                return LDPC_EINVAL;
            }
    }
    return LDPC_OK;
}

}  // namespace

extern "C" {

int ldpc_mc_run(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list, int n, int k, int dv,
                int dc, int channel, float param, int algo, float alpha, int early_stop, uint64_t seed,
                int max_iters, int expurgation, int64_t num_tests, int64_t stop_frame_errors, int batch,
                double time_limit_s, const int *devices, int ndev, int64_t *counters, int64_t *rounds) {
    int rc = check_common(channel, max_iters, batch, devices, ndev, counters);
    if (rc) return rc;
    Run r;
    r.ensemble = (variable_to_check_list == nullptr && check_to_variable_list == nullptr);
    if (r.ensemble && channel != LDPC_CH_BEC) {
        set_error("ldpc_mc_run: ensemble mode (NULL edge lists) is defined for the BEC");
        return LDPC_EINVAL;
    }
    if (!r.ensemble && (!variable_to_check_list || !check_to_variable_list)) {
        set_error("ldpc_mc_run: give both edge lists (fixed code) or neither (ensemble)");
        return LDPC_EINVAL;
    }
    r.v2c = variable_to_check_list;
    r.c2v = check_to_variable_list;
    r.n = n; r.k = k; r.dv = dv; r.dc = dc;
    r.channel = channel; r.param = param; r.algo = algo; r.alpha = alpha; r.early_stop = early_stop;
    r.seed = seed; r.max_iters = max_iters; r.expurgation = expurgation; r.batch = batch;
    std::lock_guard<std::mutex> lk(g_run_mu);
    return run_impl(r, num_tests, stop_frame_errors, time_limit_s, devices, ndev, counters, rounds);
}

int ldpc_mc_run_csr(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                    const int32_t *var_slot, int n, int m, int channel, float param, int algo, float alpha,
                    int early_stop, uint64_t seed, int max_iters, int expurgation, int64_t num_tests,
                    int64_t stop_frame_errors, int batch, double time_limit_s, const int *devices, int ndev,
                    int64_t *counters, int64_t *rounds) {
    int rc = check_common(channel, max_iters, batch, devices, ndev, counters);
    if (rc) return rc;
    if (!check_ptr || !check_var || !var_ptr || !var_slot) {
        set_error("ldpc_mc_run_csr: null CSR array");
        return LDPC_EINVAL;
    }
    Run r;
    r.cptr = check_ptr; r.cvar = check_var; r.vptr = var_ptr; r.vslot = var_slot;
    r.n = n; r.m = m;
    r.channel = channel; r.param = param; r.algo = algo; r.alpha = alpha; r.early_stop = early_stop;
    r.seed = seed; r.max_iters = max_iters; r.expurgation = expurgation; r.batch = batch;
    std::lock_guard<std::mutex> lk(g_run_mu);
    return run_impl(r, num_tests, stop_frame_errors, time_limit_s, devices, ndev, counters, rounds);
}

int ldpc_debug_mc_plan(const uint8_t *frame_error, int64_t num_trials, int64_t num_tests, int64_t stop_frame_errors,
                       int batch, int ndev, int64_t *out) {
    if (!out || (num_trials > 0 && !frame_error) || num_trials < 0 || batch <= 0 || ndev <= 0) {
        set_error("ldpc_debug_mc_plan: need out[3], the trial sequence, batch > 0, ndev > 0");
        return LDPC_EINVAL;
    }
    McPlan P;
    P.num_tests = num_tests;
    P.stop = stop_frame_errors;
    P.batch = batch;
    P.ndev = ndev;
    SeqBackend be;
    be.fe = frame_error;
    be.avail = num_trials;
    be.batch = batch;
    be.ndev = ndev;
    int64_t rounds = 0;
    const int rc = mc_drive(P, be, 0.0, rounds);
    out[0] = be.G[0];
    out[1] = be.G[1];
    out[2] = rounds;
    return rc;
}

}  // extern "C"
