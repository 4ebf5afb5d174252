// precompute_local -- drop-in for precompute_local_threads.cpp (a1-a5; the
// run_test_precompute.sh stage `./precompute_local 8`).
//   :230-250 load movielens/*.validate -> users[uimax - uid][movie]
//   :253-293 load out_fin_* -> item weights (directed, as parsed; last duplicate wins)
//   :100-213 compute_eigens per user  -> cf_eigen_batch_stream (HIP, one workgroup per user,
//            users in memory-bounded chunks)
//   :196-211 append "uid k m / evals / evecs" records to out_eigen_ (truncated first), chunk
//            by chunk as they complete (:89-98)
// Differences (documented in DESIGN.md): the item graph is dense over the compact id
// space of all ids seen (the reference's 2000x2000 matrix is only defined for ids
// < 2000); users are written in ascending uid order with their movies ascending (the
// reference's order is boost::unordered_map order); k <= 192 runs on the LDS path,
// larger k on the fp64 spill path (HBM workspace; no k cap, above CF_SPILL_MAX_K = 5000 in its
// HUGE layout).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <stdexcept>

#include "cf_cli.hpp"

int main(int argc, char** argv) {
    if (argc < 2) {   // (:217-220)
        std::printf("Usage:\n%s n_threads\n", argv[0]);
        return 1;
    }
    const std::string out_path = cfcli::opt(argc, argv, "output", "out_eigen_");
    std::map<uint32_t, std::map<uint32_t, double>> users;
    for (const auto& path : cfio::files_with_suffix("movielens/", ".validate")) {
        std::printf("Reading file: %s\n", path.c_str());
        std::string text = cfio::read_file(path);
        size_t pos = 0;
        while (pos < text.size()) {
            size_t nl = text.find('\n', pos);
            if (nl == std::string::npos) nl = text.size();
            unsigned long u, m;
            double r;
            if (std::sscanf(text.c_str() + pos, "%lu %lu %lf", &u, &m, &r) >= 2)
                users[cfio::kUimax - (uint32_t)u][(uint32_t)m] = r;
            pos = nl + 1;
        }
    }
    auto edges = cfio::load_edges(".", "out_fin_");
    std::ofstream(out_path, std::ofstream::out).close();   // truncate (:289-290)
    std::vector<uint32_t> all;
    for (auto& e : edges) {
        all.push_back(e.a);
        all.push_back(e.b);
    }
    for (auto& kv : users)
        for (auto& mr : kv.second) all.push_back(mr.first);
    cfio::IdMap items;
    items.build(all);
    std::printf("Number of movies: %u\nNumber of users: %zu\n", items.size(), users.size());

    const uint32_t n_users = (uint32_t)users.size();
    std::vector<uint64_t> off(n_users + 1, 0);
    std::vector<uint32_t> uid(n_users), its, movies;
    uint32_t u = 0;
    for (auto& kv : users) {
        uid[u] = kv.first;
        for (auto& mr : kv.second) {   // ascending movie id == ascending compact id
            its.push_back(items.at[mr.first]);
            movies.push_back(mr.first);
        }
        off[++u] = its.size();   // no k cap: k > CF_SPILL_MAX_K runs the spill path's HUGE layout
    }
    // --devices N (or CF_DEVICES): contexts on GPUs (i % visible) taking the chunks in turn
    const char* env_dev = std::getenv("CF_DEVICES");
    const int n_dev = std::max(1, std::atoi(cfcli::opt(argc, argv, "devices", env_dev ? env_dev : "1").c_str()));
    const int visible = cf_device_count();
    if (visible <= 0) cfcli::die("no usable MI355X device");
    const char* dev0 = std::getenv("CF_DEVICE");
    const int base = dev0 ? std::atoi(dev0) : 0;
    std::vector<cf_ctx*> ctxs(n_dev, nullptr);
    for (int d = 0; d < n_dev; ++d) {
        if (cf_create((base + d) % visible, &ctxs[d]) != CF_OK) cfcli::die("cf_create failed");
        cfcli::upload_edges(ctxs[d], items, edges);
    }
    // out_eigen_: records appended chunk by chunk as they complete, in user order, like the
    // reference's save_output appends each task's record (:89-98): memory is bounded by the
    // chunk size, not by the user count.  Text records are formatted on the reference's
    // n_threads (its first argument, :217-222), or the binary form with --format binary
    // (SURVEY 8f item 1).  --chunk-bytes caps a chunk's eigenvector slots (0 = by free HBM and
    // host RAM); the file is the same for every chunk size and device count.
    const int n_threads = std::max(1, std::atoi(argv[1]));
    const bool binary = cfcli::opt(argc, argv, "format", "text") == "binary";
    const uint64_t chunk_bytes = std::strtoull(cfcli::opt(argc, argv, "chunk-bytes", "0").c_str(), nullptr, 10);
    cfio::start_eigen_file(out_path, binary, n_users);
    struct Sink {
        const std::string* path;
        int n_threads;
        bool binary;
        const uint32_t* uid;
        const uint64_t* off;
        const uint32_t* movies;
    } sk{&out_path, n_threads, binary, uid.data(), off.data(), movies.data()};
    auto sink = [](void* user, const cf_eigen_chunk* c) -> int {
        const Sink& S = *static_cast<const Sink*>(user);
        try {
            cfio::write_eigen_file(*S.path, true, S.n_threads, S.binary, c->count, S.uid + c->first, c->item_off, c->m,
                                   S.movies + S.off[c->first], c->sigs, c->evals, c->packed_off, c->evecs);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "error: %s\n", e.what());
            return -1;
        }
        return 0;
    };
    cf_eigen_stream_stats st{};
    cfcli::check(ctxs[0], cf_eigen_batch_stream(ctxs.data(), n_dev, n_users, off.data(), its.data(), chunk_bytes, sink,
                                                &sk, &st),
                 "cf_eigen_batch_stream");
    std::printf("eigen stream: %u chunks of <= %.3f GB of slots (largest %.3f GB) on %d device(s); peak device "
                "memory %.3f GB own, %.3f GB in use on the device\n",
                st.chunks, st.chunk_slot_bytes / 1e9, st.max_chunk_slot_bytes / 1e9, n_dev, st.own_peak_bytes / 1e9,
                st.device_peak_bytes / 1e9);
    for (auto* c : ctxs) cf_destroy(c);
    std::printf("Wrote %u eigen records to %s\n", n_users, out_path.c_str());
    return 0;
}
