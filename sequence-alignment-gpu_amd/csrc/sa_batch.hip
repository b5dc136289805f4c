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
//     upload, one plan (sa_plan_*: one fill launch + one traceback launch for all its pairs), and
//     copy its aligned-string arenas back into the caller's per-pair buffers;
//   * the exchange step: every shard's sa_result array is gathered to device 0 with RCCL
//     (ncclGather over xGMI, one communicator per device from ncclCommInitAll) and copied to the
//     caller's results from there. Shards that share a device (num_gpus > device count, a test
//     mode for one-GPU machines) skip RCCL and copy their results directly.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
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

struct Shard {
    std::vector<int64_t> idx;  // global pair indices, in ascending order
    int device = 0;
    int rc = SA_OK;
    std::string err;
    std::vector<sa_result> res;
    sa_result *d_send = nullptr;  // RCCL send buffer (width entries)
};

// Runs one shard on its device: upload, plan, fill, traceback, strings back to the caller.
void run_shard(const sa_params *P, const sa_host_pair *pairs, Shard &sh, char *const *at, char *const *ap,
               size_t width, bool rccl)
{
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
    hipStream_t st = nullptr;
    char *dt = nullptr, *dp = nullptr;
    sa_plan *plan = nullptr;
    auto cleanup = [&]() {
        if (plan) sa_plan_destroy(plan);
        if (dt) (void)hipFree(dt);
        if (dp) (void)hipFree(dp);
        if (st) (void)hipStreamDestroy(st);
    };
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&dt, ht.size()) != hipSuccess || hipMalloc((void **)&dp, hpat.size()) != hipSuccess)
    {
        (void)hipGetLastError();
        cleanup();
        return bad(SA_ERR_NOMEM, "sa_align_batch: device allocation failed");
    }
    int rc = SA_OK;
    if (hipMemcpyAsync(dt, ht.data(), ht.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(dp, hpat.data(), hpat.size(), hipMemcpyHostToDevice, st) != hipSuccess)
        rc = SA_ERR_HIP;
    if (!rc) rc = sa_plan_create(P, pp.data(), (int64_t)k, sh.device, &plan);
    if (!rc) rc = sa_plan_fill(plan, dt, dp, st);
    if (!rc) rc = sa_plan_traceback(plan, st);
    if (!rc && rccl)
    {
        // the shard's results into the fixed-width RCCL send buffer (unused entries stay zero)
        if (hipMemsetAsync(sh.d_send, 0, width * sizeof(sa_result), st) != hipSuccess ||
            (k && hipMemcpyAsync(sh.d_send, sa_plan_device_results(plan), k * sizeof(sa_result),
                                 hipMemcpyDeviceToDevice, st) != hipSuccess))
            rc = SA_ERR_HIP;
    }
    if (!rc)
    {
        const uint64_t nb = sa_plan_output_bytes(plan);
        const bool strings = at || ap;
        std::vector<char> ot(strings ? nb : 0), op(strings ? nb : 0);
        std::vector<uint64_t> off(std::max<size_t>(1, k));
        sh.res.resize(std::max<size_t>(1, k));
        rc = sa_plan_fetch_all(plan, sh.res.data(), strings ? ot.data() : nullptr, strings ? op.data() : nullptr,
                               nb, off.data(), st);
        sh.res.resize(k);
        for (size_t q = 0; !rc && strings && q < k; ++q)
        {
            const int64_t i = sh.idx[q];
            const uint64_t L = sh.res[q].num_alignment_bytes;
            if (at && at[i] && L) std::memcpy(at[i], &ot[off[q]], L);
            if (ap && ap[i] && L) std::memcpy(ap[i], &op[off[q]], L);
        }
    }
    if (rc) bad(rc, sa_last_error());
    cleanup();
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
    // RCCL only across distinct devices (one communicator per device)
    const bool rccl = G > 1 && G <= ndev;
    std::vector<ncclComm_t> comms;
    sa_result *d_gather = nullptr;
    auto release = [&]() {
        for (ncclComm_t c : comms) (void)ncclCommDestroy(c);
        for (Shard &x : sh)
            if (x.d_send)
            {
                (void)hipSetDevice(x.device);
                (void)hipFree(x.d_send);
            }
        if (d_gather)
        {
            (void)hipSetDevice(0);
            (void)hipFree(d_gather);
        }
        (void)hipSetDevice(cur);
    };
    if (rccl)
    {
        std::vector<int> devs(G);
        for (int s = 0; s < G; ++s) devs[s] = s;
        comms.resize(G);
        if (ncclCommInitAll(comms.data(), G, devs.data()) != ncclSuccess)
        {
            comms.clear();
            release();
            return fail_b(SA_ERR_HIP, "sa_align_batch: ncclCommInitAll failed");
        }
        for (int s = 0; s < G; ++s)
        {
            (void)hipSetDevice(s);
            if (hipMalloc((void **)&sh[s].d_send, width * sizeof(sa_result)) != hipSuccess)
            {
                (void)hipGetLastError();
                release();
                return fail_b(SA_ERR_NOMEM, "sa_align_batch: RCCL buffer allocation failed");
            }
        }
        (void)hipSetDevice(0);
        if (hipMalloc((void **)&d_gather, (size_t)G * width * sizeof(sa_result)) != hipSuccess)
        {
            (void)hipGetLastError();
            release();
            return fail_b(SA_ERR_NOMEM, "sa_align_batch: RCCL buffer allocation failed");
        }
    }
    std::vector<std::thread> th;
    for (int s = 0; s < G; ++s)
        th.emplace_back(run_shard, P, pairs, std::ref(sh[s]), aligned_text, aligned_pattern, width, rccl);
    for (std::thread &t : th) t.join();
    for (const Shard &x : sh)
        if (x.rc)
        {
            release();
            return fail_b(x.rc, "sa_align_batch: shard on device " + std::to_string(x.device) + ": " + x.err);
        }
    if (rccl)
    {
        // the path's exchange step: every shard's results to device 0 (ncclGather, xGMI), one group
        std::vector<hipStream_t> streams(G, nullptr);
        bool ok = true;
        for (int s = 0; s < G && ok; ++s)
        {
            (void)hipSetDevice(s);
            ok = hipStreamCreateWithFlags(&streams[s], hipStreamNonBlocking) == hipSuccess;
        }
        ok = ok && ncclGroupStart() == ncclSuccess;
        for (int s = 0; s < G && ok; ++s)
            ok = ncclGather(sh[s].d_send, s == 0 ? d_gather : nullptr, width * sizeof(sa_result), ncclUint8, 0,
                            comms[s], streams[s]) == ncclSuccess;
        ok = (ncclGroupEnd() == ncclSuccess) && ok;
        std::vector<sa_result> all((size_t)G * width);
        if (ok)
        {
            (void)hipSetDevice(0);
            ok = hipMemcpyAsync(all.data(), d_gather, all.size() * sizeof(sa_result), hipMemcpyDeviceToHost,
                                streams[0]) == hipSuccess;
            for (int s = 0; s < G && ok; ++s)
            {
                (void)hipSetDevice(s);
                ok = hipStreamSynchronize(streams[s]) == hipSuccess;
            }
        }
        for (int s = 0; s < G; ++s)
            if (streams[s])
            {
                (void)hipSetDevice(s);
                (void)hipStreamDestroy(streams[s]);
            }
        if (!ok)
        {
            release();
            return fail_b(SA_ERR_HIP, "sa_align_batch: RCCL result gather failed");
        }
        for (int s = 0; s < G; ++s)
            for (size_t q = 0; q < sh[s].idx.size(); ++q) results[sh[s].idx[q]] = all[(size_t)s * width + q];
    }
    else
    {
        for (const Shard &x : sh)
            for (size_t q = 0; q < x.idx.size(); ++q) results[x.idx[q]] = x.res[q];
    }
    release();
    return SA_OK;
}

}  // extern "C"
