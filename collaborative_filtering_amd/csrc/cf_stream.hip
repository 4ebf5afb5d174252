// cf_stream.hip -- compute_eigens over any number of users at bounded memory.
//
// The reference schedules one compute_eigens task per user on a thread pool
// (precompute_local_threads.cpp:306-314) and each task appends its record to out_eigen_ as it
// finishes (save_output, :89-98): memory per user is constant however many users there are.
// A batched device call instead needs every user's k*max(k,2) eigenvector slot at once (the
// BASELINE config-5 set: ~250 GB of slots), so here the users are cut, in input order, into
// chunks whose slots fit a budget; each chunk is solved by the same eigen kernels, packed to
// its k x m blocks on the device (cf_pack_eigen_run), copied to pinned host memory and handed
// to the caller's sink in user order while the GPU already solves the next chunk.  Several
// contexts (GPUs) take the chunks in turn; the sink still sees them in order.  The records are
// exactly those of one cf_eigen_batch over all users: every user's result depends only on its
// own items and the graph.

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include <unistd.h>

#include "cf_internal.h"

namespace {

struct StreamChunk {
    uint32_t u0, n;
};

// Host staging of one chunk in flight (pinned): the device's outputs and the chunk-local offsets.
struct HostSet {
    int32_t* m = nullptr;
    float* sig = nullptr;
    float* eval = nullptr;
    uint64_t* poff = nullptr;    // packed offsets, count + 1
    uint64_t* off = nullptr;     // chunk-local item offsets, count + 1
    float* pack = nullptr;
    void free_all() {
        for (void* p : {(void*)m, (void*)sig, (void*)eval, (void*)poff, (void*)off, (void*)pack})
            if (p) (void)hipHostFree(p);
        m = nullptr;
        sig = eval = pack = nullptr;
        poff = off = nullptr;
    }
};

struct StreamState {
    std::vector<StreamChunk> chunks;
    std::vector<HostSet> sets;
    std::vector<int> ready;          // per chunk: 0 pending, 1 staged, -1 failed
    uint32_t delivered = 0;          // chunks handed to the sink
    std::atomic<uint32_t> next{0};   // next chunk a worker claims
    std::atomic<bool> stop{false};
    std::mutex mu;
    std::condition_variable cv;
};

struct WorkerStats {
    uint64_t own_peak = 0;       // the stream's device buffers + the context's workspaces
    uint64_t device_peak = 0;    // device-wide bytes in use (total - free) after a chunk's solve
    uint32_t chunks = 0;
};

uint64_t host_ram_bytes() {
    const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGE_SIZE);
    return (pages > 0 && psz > 0) ? (uint64_t)pages * (uint64_t)psz : (16ull << 30);
}

int stream_worker(cf_ctx* ctx, StreamState& S, const uint64_t* item_off, const uint32_t* items,
                  uint32_t max_users, uint64_t max_entries, uint64_t max_slots, WorkerStats& st) {
    CF_TRY(set_device(ctx));
    hipStream_t stream = nullptr;
    CF_HIP_CHECK(ctx, hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    struct StreamGuard {
        hipStream_t s;
        ~StreamGuard() {
            if (s) (void)hipStreamDestroy(s);
        }
    } guard{stream};
    DevBuf d_off, d_items, d_eoff, d_m, d_sig, d_eval, d_evec, d_poff, d_pack;
    const uint64_t mu = std::max<uint64_t>(max_users, 1), me = std::max<uint64_t>(max_entries, 1);
    CF_TRY(dev_alloc(ctx, d_off, sizeof(uint64_t) * (mu + 1)));
    CF_TRY(dev_alloc(ctx, d_items, sizeof(uint32_t) * me));
    CF_TRY(dev_alloc(ctx, d_eoff, sizeof(uint64_t) * mu));
    CF_TRY(dev_alloc(ctx, d_m, sizeof(int32_t) * mu));
    CF_TRY(dev_alloc(ctx, d_sig, sizeof(float) * me));
    CF_TRY(dev_alloc(ctx, d_eval, sizeof(float) * me));
    CF_TRY(dev_alloc(ctx, d_evec, sizeof(float) * std::max<uint64_t>(max_slots, 1)));
    CF_TRY(dev_alloc(ctx, d_poff, sizeof(uint64_t) * (mu + 1)));
    CF_TRY(dev_alloc(ctx, d_pack, sizeof(float) * std::max<uint64_t>(max_slots, 1)));
    const uint64_t own = sizeof(uint64_t) * (mu + 1) * 2 + sizeof(uint32_t) * me + sizeof(uint64_t) * mu +
                         sizeof(int32_t) * mu + 2 * sizeof(float) * me + 2 * sizeof(float) * std::max<uint64_t>(max_slots, 1);
    std::vector<uint64_t> eoff(mu);
    const uint32_t n_sets = (uint32_t)S.sets.size();
    for (;;) {
        if (S.stop.load()) return CF_OK;
        const uint32_t c = S.next.fetch_add(1);
        if (c >= S.chunks.size()) return CF_OK;
        {   // the host set of chunk c is free once chunk c - n_sets has been delivered
            std::unique_lock<std::mutex> lk(S.mu);
            S.cv.wait(lk, [&] { return S.stop.load() || S.delivered + n_sets > c; });
            if (S.stop.load()) return CF_OK;
        }
        const StreamChunk& ch = S.chunks[c];
        HostSet& H = S.sets[c % n_sets];
        const uint64_t e0 = item_off[ch.u0], ne = item_off[ch.u0 + ch.n] - e0;
        for (uint32_t u = 0; u <= ch.n; ++u) H.off[u] = item_off[ch.u0 + u] - e0;
        const uint64_t n_evec = cf_evec_offsets(ch.n, H.off, eoff.data());
        if (n_evec > max_slots || ne > max_entries || ch.n > max_users)
            return cf_set_error(ctx, CF_EINVAL, "eigen stream: chunk larger than its buffers");
        cf_plan* plan = nullptr;
        CF_TRY(cf_plan_create(ctx, ch.n, H.off, &plan));
        struct PlanGuard {
            cf_plan* p;
            ~PlanGuard() { cf_plan_destroy(p); }
        } pg{plan};
        CF_HIP_CHECK(ctx, hipMemcpyAsync(d_off.p, H.off, sizeof(uint64_t) * (ch.n + 1), hipMemcpyHostToDevice, stream));
        if (ne) CF_HIP_CHECK(ctx, hipMemcpyAsync(d_items.p, items + e0, sizeof(uint32_t) * ne, hipMemcpyHostToDevice, stream));
        CF_HIP_CHECK(ctx, hipMemcpyAsync(d_eoff.p, eoff.data(), sizeof(uint64_t) * ch.n, hipMemcpyHostToDevice, stream));
        CF_HIP_CHECK(ctx, hipMemsetAsync(d_eval.p, 0, sizeof(float) * std::max<uint64_t>(ne, 1), stream));
        CF_TRY(cf_launch_eigen(ctx, plan, (const uint64_t*)d_off.p, (const uint32_t*)d_items.p,
                               (const uint64_t*)d_eoff.p, (int32_t*)d_m.p, (float*)d_sig.p, (float*)d_eval.p,
                               (float*)d_evec.p, stream));
        CF_TRY(cf_pack_eigen_run(ctx, ch.n, (const uint64_t*)d_off.p, (const int32_t*)d_m.p, (const uint64_t*)d_eoff.p,
                                 (const float*)d_evec.p, (uint64_t*)d_poff.p, (float*)d_pack.p, stream));
        CF_HIP_CHECK(ctx, hipMemcpyAsync(H.m, d_m.p, sizeof(int32_t) * ch.n, hipMemcpyDeviceToHost, stream));
        CF_HIP_CHECK(ctx, hipMemcpyAsync(H.poff, d_poff.p, sizeof(uint64_t) * (ch.n + 1), hipMemcpyDeviceToHost, stream));
        if (ne) {
            CF_HIP_CHECK(ctx, hipMemcpyAsync(H.sig, d_sig.p, sizeof(float) * ne, hipMemcpyDeviceToHost, stream));
            CF_HIP_CHECK(ctx, hipMemcpyAsync(H.eval, d_eval.p, sizeof(float) * ne, hipMemcpyDeviceToHost, stream));
        }
        CF_HIP_CHECK(ctx, hipStreamSynchronize(stream));
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
            st.device_peak = std::max<uint64_t>(st.device_peak, (uint64_t)(total_b - free_b));
        st.own_peak = std::max<uint64_t>(st.own_peak, own + ctx->spill_bytes + ctx->tri_bytes + ctx->scratch_bytes);
        const uint64_t packed = H.poff[ch.n];
        if (packed > n_evec) return cf_set_error(ctx, CF_EHIP, "eigen stream: packed size exceeds the slots");
        if (packed) {
            CF_HIP_CHECK(ctx, hipMemcpyAsync(H.pack, d_pack.p, sizeof(float) * packed, hipMemcpyDeviceToHost, stream));
            CF_HIP_CHECK(ctx, hipStreamSynchronize(stream));
        }
        ++st.chunks;
        {
            std::lock_guard<std::mutex> lk(S.mu);
            S.ready[c] = 1;
        }
        S.cv.notify_all();
    }
}

}  // namespace

extern "C" {

int cf_eigen_batch_stream(cf_ctx* const* ctxs, int n_dev, uint32_t n_users, const uint64_t* item_off,
                          const uint32_t* items, uint64_t chunk_bytes, cf_eigen_sink sink, void* sink_user,
                          cf_eigen_stream_stats* stats) {
    if (!ctxs || n_dev <= 0 || !ctxs[0]) return CF_EINVAL;
    cf_ctx* root = ctxs[0];
    if (!item_off || (item_off[n_users] && !items) || !sink)
        return cf_set_error(root, CF_EINVAL, "cf_eigen_batch_stream: null argument");
    for (int d = 0; d < n_dev; ++d) {
        if (!ctxs[d]) return cf_set_error(root, CF_EINVAL, "cf_eigen_batch_stream: null context");
        if (!has_graph(ctxs[d])) return cf_set_error(root, CF_ESTATE, "cf_eigen_batch_stream: a context has no graph");
        for (int e = 0; e < d; ++e)
            if (ctxs[e] == ctxs[d]) return cf_set_error(root, CF_EINVAL, "cf_eigen_batch_stream: a context appears twice");
    }
    for (uint32_t u = 0; u < n_users; ++u)
        if (item_off[u + 1] < item_off[u]) return cf_set_error(root, CF_EINVAL, "cf_eigen_batch_stream: item_off decreases");
    const uint64_t n_entries = item_off[n_users];
    for (int d = 0; d < n_dev; ++d)
        for (uint64_t e = 0; e < n_entries; ++e)
            if (items[e] >= ctxs[d]->n_items) return cf_set_error(root, CF_EINVAL, "item index outside the graph");
    if (stats) *stats = cf_eigen_stream_stats{};
    // chunk budget (eigenvector-slot bytes): the caller's, else the smaller of a fifth of the
    // device share (the slots and their packed copy; the spill workspace sizes itself from what
    // is left) and the pinned host staging share (2 sets per device in flight)
    const uint32_t n_sets = 2u * (uint32_t)n_dev;
    uint64_t cap = chunk_bytes;
    if (cap == 0) {
        CF_TRY(set_device(root));
        const uint64_t dev_cap = cf_hbm_budget(root, 0, 0.2, 1ull << 30);
        const uint64_t host_cap = std::min<uint64_t>(host_ram_bytes() / 4, 64ull << 30) / n_sets;
        cap = std::max<uint64_t>(std::min(dev_cap, host_cap), 64ull << 20);
    }
    const uint64_t cap_floats = std::max<uint64_t>(cap / sizeof(float), 1);
    StreamState S;
    uint32_t max_users = 0;
    uint64_t max_entries = 0, max_slots = 0;
    for (uint32_t u = 0; u < n_users;) {   // contiguous, >= 1 user, slots within the budget
        uint32_t v = u;
        uint64_t slots = 0;
        while (v < n_users) {
            const uint64_t s = cf_evec_slots((uint32_t)(item_off[v + 1] - item_off[v]));
            if (v > u && slots + s > cap_floats) break;
            slots += s;
            ++v;
        }
        S.chunks.push_back({u, v - u});
        max_users = std::max(max_users, v - u);
        max_entries = std::max<uint64_t>(max_entries, item_off[v] - item_off[u]);
        max_slots = std::max(max_slots, slots);
        u = v;
    }
    S.ready.assign(S.chunks.size(), 0);
    const uint32_t sets = std::min<uint32_t>(n_sets, std::max<uint32_t>((uint32_t)S.chunks.size(), 1));
    S.sets.resize(sets);
    int rc = CF_OK;
    for (HostSet& H : S.sets) {
        const uint64_t mu = std::max<uint32_t>(max_users, 1), me = std::max<uint64_t>(max_entries, 1);
        if (hipHostMalloc((void**)&H.m, sizeof(int32_t) * mu) != hipSuccess ||
            hipHostMalloc((void**)&H.sig, sizeof(float) * me) != hipSuccess ||
            hipHostMalloc((void**)&H.eval, sizeof(float) * me) != hipSuccess ||
            hipHostMalloc((void**)&H.poff, sizeof(uint64_t) * (mu + 1)) != hipSuccess ||
            hipHostMalloc((void**)&H.off, sizeof(uint64_t) * (mu + 1)) != hipSuccess ||
            hipHostMalloc((void**)&H.pack, sizeof(float) * std::max<uint64_t>(max_slots, 1)) != hipSuccess) {
            (void)hipGetLastError();
            rc = cf_set_error(root, CF_ENOMEM, "cf_eigen_batch_stream: pinned staging (" +
                                                   std::to_string(4 * max_slots) + " bytes per set)");
            break;
        }
    }
    std::vector<WorkerStats> ws(n_dev);
    std::vector<int> wrc(n_dev, CF_OK);
    std::vector<std::thread> pool;
    if (rc == CF_OK)
        for (int d = 0; d < n_dev; ++d)
            pool.emplace_back([&, d] {
                wrc[d] = stream_worker(ctxs[d], S, item_off, items, max_users, max_entries, max_slots, ws[d]);
                if (wrc[d] != CF_OK) {
                    std::lock_guard<std::mutex> lk(S.mu);
                    S.stop = true;
                }
                S.cv.notify_all();
            });
    // deliver in order: chunk c once staged by whichever device solved it
    for (uint32_t c = 0; rc == CF_OK && c < S.chunks.size(); ++c) {
        {
            std::unique_lock<std::mutex> lk(S.mu);
            S.cv.wait(lk, [&] { return S.ready[c] != 0 || S.stop.load(); });
            if (S.ready[c] != 1) break;   // a worker failed
        }
        const StreamChunk& ch = S.chunks[c];
        const HostSet& H = S.sets[c % S.sets.size()];
        cf_eigen_chunk out;
        out.first = ch.u0;
        out.count = ch.n;
        out.item_off = H.off;
        out.m = H.m;
        out.sigs = H.sig;
        out.evals = H.eval;
        out.packed_off = H.poff;
        out.evecs = H.pack;
        const int src = sink(sink_user, &out);
        if (src != 0) {
            rc = cf_set_error(root, src < 0 ? src : CF_EINVAL, "cf_eigen_batch_stream: the sink stopped the call at chunk " +
                                                                 std::to_string(c));
            std::lock_guard<std::mutex> lk(S.mu);
            S.stop = true;
        }
        {
            std::lock_guard<std::mutex> lk(S.mu);
            S.delivered = c + 1;
        }
        S.cv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(S.mu);
        if (rc != CF_OK) S.stop = true;
    }
    S.cv.notify_all();
    for (auto& t : pool) t.join();
    for (int d = 0; d < n_dev && rc == CF_OK; ++d)
        if (wrc[d] != CF_OK) rc = cf_set_error(root, wrc[d], "device part " + std::to_string(d) + ": " + ctxs[d]->last_error);
    if (rc == CF_OK && S.delivered != S.chunks.size()) rc = cf_set_error(root, CF_EHIP, "cf_eigen_batch_stream: chunks lost");
    for (HostSet& H : S.sets) H.free_all();
    // one-shot call: the contexts' eigen workspaces (the spill solver's may hold 3/4 of the
    // device share) are not kept for a next call
    for (int d = 0; d < n_dev; ++d) {
        (void)hipSetDevice(ctxs[d]->device);
        (void)cf_evict_workspaces(ctxs[d]);
    }
    (void)hipSetDevice(root->device);
    if (stats) {
        stats->chunks = (uint32_t)S.chunks.size();
        stats->chunk_slot_bytes = cap;
        for (int d = 0; d < n_dev; ++d) {
            stats->own_peak_bytes = std::max(stats->own_peak_bytes, ws[d].own_peak);
            stats->device_peak_bytes = std::max(stats->device_peak_bytes, ws[d].device_peak);
        }
        stats->max_chunk_slot_bytes = 4 * max_slots;
    }
    return rc;
}

}  // extern "C"
