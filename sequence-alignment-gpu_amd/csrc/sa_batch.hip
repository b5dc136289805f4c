// sa_align_batch — many independent pairs from host memory, sharded over the node's GPUs, in one
// process (BASELINE.json config 5; SURVEY.md §8(b) proposed C ABI, §8(e) partitioning).
//
// The reference has no multi-GPU path; its batch caller aligns requests one after another on
// device 0 (tests/benchmarks.cu:271-332). Here:
//   * the deal (sa_batch_deal): equal-work pairs go round-robin, pair i -> shard i mod G (as
//     sa_amd.distributed.shard does for the torch path); unequal pairs by longest-processing-time
//     (largest n*m first, to the least-loaded shard, ties to the lower shard), so shards finish
//     together;
//   * one host thread per shard: pack the shard's inputs into one text and one pattern arena,
//     upload, one plan (sa_plan_*: one fill launch + one traceback launch for all its pairs), its
//     sa_result array into a fixed-width RCCL send buffer, its aligned-string arenas to the host;
//   * the exchange step: every shard's sa_result array is gathered to device 0 with RCCL
//     (ncclGather over xGMI) and the caller's results come from that gathered buffer only; the
//     strings are copied into the caller's buffers after it, with the gathered lengths. RCCL is
//     loaded on first use (dlopen: callers that never shard over several devices do not need it)
//     and the communicators of a device set are created once per process (and dropped after a failed
//     gather, so the next call rebuilds them). Shards that share a device (num_gpus > device count, a
//     test mode for one-GPU machines) skip RCCL and take their results from their own plan;
//   * per shard slot, a cache that lives across calls: its stream, its device input arenas and RCCL
//     send buffer (grow-only), and its plan, reused while the shard's pair shapes and the scoring
//     parameters stay the same (a repeated batch costs its uploads, kernels and copies only), plus
//     the gather buffer on device 0. Calls are serialised process-wide (g_batch_mu).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "sa_hip.h"

namespace sa {
int set_error(int code, const std::string &msg);  // sa_engine.hip: what sa_last_error() reports
}

namespace {

int fail_b(int code, const std::string &msg) { return sa::set_error(code, msg); }

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

// ---- RCCL, loaded on first use -------------------------------------------------------------------
struct Rccl {
    bool tried = false, ok = false;
    std::string err;
    ncclResult_t (*commInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
};

std::mutex g_batch_mu;  // one sa_align_batch at a time per process (shared communicators)

Rccl &rccl()
{
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h)
    {
        const char *e = dlerror();
        r.err = std::string("cannot load librccl: ") + (e ? e : "?");
        return r;
    }
    r.commInitAll = reinterpret_cast<decltype(r.commInitAll)>(dlsym(h, "ncclCommInitAll"));
    r.groupStart = reinterpret_cast<decltype(r.groupStart)>(dlsym(h, "ncclGroupStart"));
    r.groupEnd = reinterpret_cast<decltype(r.groupEnd)>(dlsym(h, "ncclGroupEnd"));
    r.gather = reinterpret_cast<decltype(r.gather)>(dlsym(h, "ncclGather"));
    r.ok = r.commInitAll && r.groupStart && r.groupEnd && r.gather;
    if (!r.ok) r.err = "librccl lacks ncclCommInitAll / ncclGroupStart / ncclGroupEnd / ncclGather";
    return r;
}

// Communicators of devices 0..G-1, created once per process (never destroyed: RCCL tears them down
// at exit; destroying them from a static destructor can run after the HIP runtime is gone).
std::map<int, std::vector<ncclComm_t>> g_comms;

// ---- per-shard caches (across calls) ------------------------------------------------------------
struct ShardCache {
    int device = -1;
    hipStream_t st = nullptr;
    char *dt = nullptr, *dp = nullptr;  // input arenas
    size_t dt_cap = 0, dp_cap = 0;
    sa_result *d_send = nullptr;        // RCCL send buffer
    size_t send_cap = 0;
    sa_plan *plan = nullptr;            // the last plan and what it was built for
    std::vector<sa_pair> plan_pairs;
    std::vector<int32_t> plan_params;   // mode, A, gap, rows_per_lane, the matrix, the alphabet bytes
};
std::vector<ShardCache> g_cache;
sa_result *g_gather = nullptr;  // device 0
size_t g_gather_cap = 0;

void free_cache_slot(ShardCache &c)
{
    if (c.device < 0) return;
    (void)hipSetDevice(c.device);
    if (c.plan) sa_plan_destroy(c.plan);
    if (c.dt) (void)hipFree(c.dt);
    if (c.dp) (void)hipFree(c.dp);
    if (c.d_send) (void)hipFree(c.d_send);
    if (c.st) (void)hipStreamDestroy(c.st);
    c = ShardCache();
}

// atexit: a thread still inside sa_align_batch holds the lock and uses these objects, so the frees
// are skipped then (leaking at exit is harmless; blocking here would deadlock the shutdown)
void release_batch_cache()
{
    std::unique_lock<std::mutex> lock(g_batch_mu, std::try_to_lock);
    if (!lock.owns_lock()) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (ShardCache &c : g_cache) free_cache_slot(c);
    g_cache.clear();
    if (g_gather)
    {
        (void)hipSetDevice(0);
        (void)hipFree(g_gather);
    }
    g_gather = nullptr;
    g_gather_cap = 0;
    (void)hipSetDevice(cur);
}

// grow-only device buffer (contents not kept)
template <typename T>
bool ensure(T **p, size_t &cap, size_t bytes)
{
    if (cap >= bytes && *p) return true;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    if (hipMalloc((void **)p, bytes) != hipSuccess)
    {
        (void)hipGetLastError();
        *p = nullptr;
        return false;
    }
    cap = bytes;
    return true;
}

std::vector<int32_t> params_key(const sa_params *P)
{
    std::vector<int32_t> k{P->mode, P->alphabet_size, P->gap_penalty, P->rows_per_lane};
    for (int e = 0; e < P->alphabet_size * P->alphabet_size; ++e) k.push_back(P->score_matrix[e]);
    if (P->alphabet)
        for (int c = 0; c <= P->alphabet_size && P->alphabet[c]; ++c) k.push_back((int32_t)(unsigned char)P->alphabet[c]);
    return k;
}

bool same_pairs(const std::vector<sa_pair> &a, const std::vector<sa_pair> &b)
{
    if (a.size() != b.size()) return false;
    for (size_t q = 0; q < a.size(); ++q)
        if (a[q].text_offset != b[q].text_offset || a[q].text_len != b[q].text_len ||
            a[q].pattern_offset != b[q].pattern_offset || a[q].pattern_len != b[q].pattern_len)
            return false;
    return true;
}

// ---- shards -------------------------------------------------------------------------------------
struct Shard {
    std::vector<int64_t> idx;  // global pair indices, in ascending order
    int device = 0;
    int rc = SA_OK;
    std::string err;
    std::vector<sa_result> res;    // own results (no RCCL only)
    std::vector<char> ot, op;      // aligned-string arenas on the host
    std::vector<uint64_t> off;     // each pair's offset in the arenas
    ShardCache *c = nullptr;       // this shard's cache slot (stream, arenas, send buffer, plan)
    double ms = 0;
};

thread_local int32_t t_last_shards = 0, t_last_rccl = 0;
thread_local std::vector<double> t_last_ms;
thread_local double t_last_gather_ms = 0;

// Runs one shard on its device: upload, plan (the cached one when the shapes match), fill, traceback;
// results into the RCCL send buffer (rccl) or to the host, aligned-string arenas to the host (when the
// caller wants strings).
void run_shard(const sa_params *P, const std::vector<int32_t> &pkey, const sa_host_pair *pairs, Shard &sh,
               bool strings, size_t width, bool rccl_path)
{
    const Clock::time_point t0 = Clock::now();
    auto bad = [&](int code, const std::string &msg) {
        sh.rc = code;
        sh.err = msg;
    };
    if (hipSetDevice(sh.device) != hipSuccess) return bad(SA_ERR_HIP, "hipSetDevice failed");
    const size_t k = sh.idx.size();
    std::vector<sa_pair> pp(k);
    uint64_t tb = 0, pb = 0;
    for (size_t q = 0; q < k; ++q)
    {
        const sa_host_pair &h = pairs[sh.idx[q]];
        pp[q] = sa_pair{tb, h.text_len, pb, h.pattern_len};
        tb += h.text_len;
        pb += h.pattern_len;
    }
    std::vector<char> ht(tb + 16, 0), hpat(pb + 16, 0);
    for (size_t q = 0; q < k; ++q)
    {
        const sa_host_pair &h = pairs[sh.idx[q]];
        if (h.text_len) std::memcpy(&ht[pp[q].text_offset], h.text, h.text_len);
        if (h.pattern_len) std::memcpy(&hpat[pp[q].pattern_offset], h.pattern, h.pattern_len);
    }
    ShardCache &c = *sh.c;
    if (!ensure(&c.dt, c.dt_cap, ht.size()) || !ensure(&c.dp, c.dp_cap, hpat.size()))
        return bad(SA_ERR_NOMEM, "sa_align_batch: device allocation failed");
    int rc = SA_OK;
    if (hipMemcpyAsync(c.dt, ht.data(), ht.size(), hipMemcpyHostToDevice, c.st) != hipSuccess ||
        hipMemcpyAsync(c.dp, hpat.data(), hpat.size(), hipMemcpyHostToDevice, c.st) != hipSuccess)
        rc = SA_ERR_HIP;
    if (!rc && !(c.plan && c.plan_params == pkey && same_pairs(c.plan_pairs, pp)))
    {
        if (c.plan)
        {
            (void)hipStreamSynchronize(c.st);  // (the old plan's last kernels are done with it)
            sa_plan_destroy(c.plan);
            c.plan = nullptr;
        }
        rc = sa_plan_create(P, pp.data(), (int64_t)k, sh.device, &c.plan);
        if (!rc)
        {
            c.plan_pairs = pp;
            c.plan_params = pkey;
        }
        else c.plan = nullptr;
    }
    sa_plan *plan = c.plan;
    if (!rc) rc = sa_plan_fill(plan, c.dt, c.dp, c.st);
    if (!rc) rc = sa_plan_traceback(plan, c.st);
    if (!rc && rccl_path)
    {
        // the shard's results into the fixed-width RCCL send buffer (unused entries stay zero)
        if (hipMemsetAsync(c.d_send, 0, width * sizeof(sa_result), c.st) != hipSuccess ||
            (k && sa_plan_copy_results(plan, c.d_send, c.st) != SA_OK))
            rc = SA_ERR_HIP;
    }
    if (!rc)
    {
        const uint64_t nb = sa_plan_output_bytes(plan);
        sh.ot.assign(strings ? nb : 0, 0);
        sh.op.assign(strings ? nb : 0, 0);
        sh.off.assign(std::max<size_t>(1, k), 0);
        if (!rccl_path) sh.res.resize(std::max<size_t>(1, k));
        // (also synchronises the stream: the send buffer is complete before the gather)
        rc = sa_plan_fetch_all(plan, rccl_path ? nullptr : sh.res.data(), strings ? sh.ot.data() : nullptr,
                               strings ? sh.op.data() : nullptr, nb, sh.off.data(), c.st);
        if (!rccl_path) sh.res.resize(k);
    }
    if (rc)
    {
        bad(rc, sa_last_error());
        // a failed plan is not reused (a timed-out fill may have left it mid-way)
        (void)hipStreamSynchronize(c.st);
        if (c.plan) sa_plan_destroy(c.plan);
        c.plan = nullptr;
        c.plan_pairs.clear();
    }
    sh.ms = ms_since(t0);
}

}  // namespace

extern "C" {

int sa_batch_deal(const uint64_t *cells, int64_t num_pairs, int num_shards, int32_t *shard_of)
{
    if (num_pairs < 0 || num_shards < 1 || (num_pairs > 0 && (!cells || !shard_of)))
        return fail_b(SA_ERR_INVALID, "sa_batch_deal: bad argument");
    bool equal = true;
    for (int64_t i = 1; i < num_pairs; ++i) equal = equal && cells[i] == cells[0];
    if (equal)
    {
        for (int64_t i = 0; i < num_pairs; ++i) shard_of[i] = (int32_t)(i % num_shards);
        return SA_OK;
    }
    std::vector<int64_t> order(num_pairs);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return cells[a] > cells[b]; });
    std::vector<uint64_t> load(num_shards, 0);
    for (int64_t i : order)
    {
        const int s = (int)(std::min_element(load.begin(), load.end()) - load.begin());  // first least-loaded
        shard_of[i] = s;
        load[s] += std::max<uint64_t>(cells[i], 1);
    }
    return SA_OK;
}

int sa_batch_last_stats(int32_t *num_shards, int32_t *used_rccl, double *shard_ms, int32_t cap, double *gather_ms)
{
    if (num_shards) *num_shards = t_last_shards;
    if (used_rccl) *used_rccl = t_last_rccl;
    for (int32_t s = 0; shard_ms && s < cap && s < (int32_t)t_last_ms.size(); ++s) shard_ms[s] = t_last_ms[s];
    if (gather_ms) *gather_ms = t_last_gather_ms;
    return SA_OK;
}

int sa_align_batch(const sa_params *P, const sa_host_pair *pairs, int64_t num_pairs, int num_gpus,
                   sa_result *results, char *const *aligned_text, char *const *aligned_pattern)
{
    if (!P || num_pairs < 0 || num_gpus < 1 || (num_pairs > 0 && (!pairs || !results)))
        return fail_b(SA_ERR_INVALID, "sa_align_batch: bad argument");
    for (int64_t i = 0; i < num_pairs; ++i)
    {
        const sa_host_pair &h = pairs[i];
        if ((h.text_len && !h.text) || (h.pattern_len && !h.pattern))
            return fail_b(SA_ERR_INVALID, "sa_align_batch: null sequence");
        for (uint64_t x = 0; x < h.text_len; ++x)
            if (h.text[x] < 0 || h.text[x] >= P->alphabet_size) return fail_b(SA_ERR_INVALID, "text byte outside the alphabet");
        for (uint64_t x = 0; x < h.pattern_len; ++x)
            if (h.pattern[x] < 0 || h.pattern[x] >= P->alphabet_size) return fail_b(SA_ERR_INVALID, "pattern byte outside the alphabet");
    }
    std::lock_guard<std::mutex> lock(g_batch_mu);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail_b(SA_ERR_HIP, "no HIP device");
    int cur = 0;
    (void)hipGetDevice(&cur);
    const int G = (int)std::min<int64_t>(num_gpus, std::max<int64_t>(1, num_pairs));
    std::vector<uint64_t> cells(num_pairs);
    for (int64_t i = 0; i < num_pairs; ++i) cells[i] = pairs[i].text_len * pairs[i].pattern_len;
    std::vector<int32_t> shard_of(std::max<int64_t>(1, num_pairs));
    if (int rc = sa_batch_deal(cells.data(), num_pairs, G, shard_of.data())) return rc;
    std::vector<Shard> sh(G);
    for (int64_t i = 0; i < num_pairs; ++i) sh[shard_of[i]].idx.push_back(i);
    size_t width = 1;
    for (int s = 0; s < G; ++s)
    {
        sh[s].device = s % ndev;
        width = std::max(width, sh[s].idx.size());
    }
    t_last_shards = G;
    t_last_rccl = 0;
    t_last_ms.assign(G, 0.0);
    t_last_gather_ms = 0;
    // RCCL only across distinct devices (one communicator per device)
    const bool use_rccl = G > 1 && G <= ndev;
    auto restore = [&]() { (void)hipSetDevice(cur); };
    // the shards' cache slots (created on first use; a slot whose device changed is rebuilt); the
    // process frees them at exit (registered after HIP initialised, so it runs before its teardown)
    static bool s_atexit = false;
    if (!s_atexit)
    {
        std::atexit(release_batch_cache);
        s_atexit = true;
    }
    if (g_cache.size() < (size_t)G) g_cache.resize(G);
    for (int s = 0; s < G; ++s)
    {
        ShardCache &c = g_cache[s];
        if (c.device != sh[s].device) free_cache_slot(c);
        c.device = sh[s].device;
        sh[s].c = &c;
        (void)hipSetDevice(c.device);
        if (!c.st && hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking) != hipSuccess)
        {
            (void)hipGetLastError();
            c.st = nullptr;
            restore();
            return fail_b(SA_ERR_HIP, "sa_align_batch: stream creation failed");
        }
    }
    std::vector<ncclComm_t> *comms = nullptr;
    if (use_rccl)
    {
        Rccl &R = rccl();
        if (!R.ok)
        {
            restore();
            return fail_b(SA_ERR_HIP, "sa_align_batch: " + R.err);
        }
        auto it = g_comms.find(G);
        if (it == g_comms.end())
        {
            std::vector<int> devs(G);
            std::iota(devs.begin(), devs.end(), 0);
            std::vector<ncclComm_t> c(G);
            if (R.commInitAll(c.data(), G, devs.data()) != ncclSuccess)
            {
                restore();
                return fail_b(SA_ERR_HIP, "sa_align_batch: ncclCommInitAll failed");
            }
            it = g_comms.emplace(G, std::move(c)).first;
        }
        comms = &it->second;
        for (int s = 0; s < G; ++s)
        {
            (void)hipSetDevice(s);
            if (!ensure(&sh[s].c->d_send, sh[s].c->send_cap, width * sizeof(sa_result)))
            {
                restore();
                return fail_b(SA_ERR_NOMEM, "sa_align_batch: RCCL buffer allocation failed");
            }
        }
        (void)hipSetDevice(0);
        if (!ensure(&g_gather, g_gather_cap, (size_t)G * width * sizeof(sa_result)))
        {
            restore();
            return fail_b(SA_ERR_NOMEM, "sa_align_batch: RCCL buffer allocation failed");
        }
    }
    const bool strings = aligned_text || aligned_pattern;
    const std::vector<int32_t> pkey = params_key(P);
    std::vector<std::thread> th;
    for (int s = 0; s < G; ++s)
        th.emplace_back(run_shard, P, std::cref(pkey), pairs, std::ref(sh[s]), strings, width, use_rccl);
    for (std::thread &t : th) t.join();
    for (int s = 0; s < G; ++s) t_last_ms[s] = sh[s].ms;
    for (const Shard &x : sh)
        if (x.rc)
        {
            restore();
            return fail_b(x.rc, "sa_align_batch: shard on device " + std::to_string(x.device) + ": " + x.err);
        }
    // per-pair results: gathered over RCCL (the exchange step) or straight from each shard
    std::vector<sa_result> all;
    if (use_rccl)
    {
        const Clock::time_point tg = Clock::now();
        Rccl &R = rccl();
        bool ok = R.groupStart() == ncclSuccess;
        for (int s = 0; s < G && ok; ++s)
            ok = R.gather(sh[s].c->d_send, s == 0 ? g_gather : nullptr, width * sizeof(sa_result), ncclUint8, 0,
                          (*comms)[s], sh[s].c->st) == ncclSuccess;
        ok = (R.groupEnd() == ncclSuccess) && ok;
        all.resize((size_t)G * width);
        if (ok)
        {
            (void)hipSetDevice(0);
            ok = hipMemcpyAsync(all.data(), g_gather, all.size() * sizeof(sa_result), hipMemcpyDeviceToHost,
                                sh[0].c->st) == hipSuccess;
            for (int s = 0; s < G && ok; ++s)
            {
                (void)hipSetDevice(s);
                ok = hipStreamSynchronize(sh[s].c->st) == hipSuccess;
            }
        }
        if (!ok)
        {
            // a communicator left in an error state is not reused: the next call builds new ones
            // (the failed ones are abandoned, not destroyed: their state is unknown)
            g_comms.erase(G);
            restore();
            return fail_b(SA_ERR_HIP, "sa_align_batch: RCCL result gather failed");
        }
        t_last_gather_ms = ms_since(tg);
        t_last_rccl = 1;
    }
    for (int s = 0; s < G; ++s)
    {
        const Shard &x = sh[s];
        for (size_t q = 0; q < x.idx.size(); ++q)
        {
            const int64_t i = x.idx[q];
            results[i] = use_rccl ? all[(size_t)s * width + q] : x.res[q];
            const uint64_t L = results[i].num_alignment_bytes;
            if (aligned_text && aligned_text[i] && L) std::memcpy(aligned_text[i], &x.ot[x.off[q]], L);
            if (aligned_pattern && aligned_pattern[i] && L) std::memcpy(aligned_pattern[i], &x.op[x.off[q]], L);
        }
    }
    restore();
    return SA_OK;
}

}  // extern "C"
