// cf_cli.hpp -- shared plumbing of the drop-in stage binaries (bin_*.cpp).
#pragma once

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "cf_abi.h"
#include "cf_io.hpp"

namespace cfcli {

[[noreturn]] inline void die(const std::string& msg) {
    std::fprintf(stderr, "error: %s\n", msg.c_str());
    std::exit(1);
}

inline void check(cf_ctx* ctx, int rc, const char* what) {
    if (rc != CF_OK) die(std::string(what) + " failed (" + std::to_string(rc) + "): " + cf_last_error(ctx));
}

inline cf_ctx* open_device() {
    cf_ctx* ctx = nullptr;
    const char* dev = std::getenv("CF_DEVICE");
    const int rc = cf_create(dev ? std::atoi(dev) : 0, &ctx);
    if (rc != CF_OK) die("cf_create failed (" + std::to_string(rc) + "): no usable MI355X device");
    return ctx;
}

// Upload a directed edge list over a compact id space as the context's item graph.
inline void upload_edges(cf_ctx* ctx, const cfio::IdMap& ids, const std::vector<cfio::Edge>& edges) {
    const uint32_t n = ids.size();
    std::vector<uint64_t> row_ptr(n + 1, 0);
    for (const auto& e : edges) row_ptr[ids.at.at(e.a) + 1]++;
    for (uint32_t i = 0; i < n; ++i) row_ptr[i + 1] += row_ptr[i];
    std::vector<uint32_t> col(edges.size());
    std::vector<float> w(edges.size());
    std::vector<uint64_t> fill(row_ptr.begin(), row_ptr.end() - 1);
    for (const auto& e : edges) {   // file order within a row: the last duplicate wins
        const uint64_t p = fill[ids.at.at(e.a)]++;
        col[p] = ids.at.at(e.b);
        w[p] = (float)e.w;
    }
    check(ctx, cf_item_graph_upload(ctx, n, row_ptr.data(), col.data(), w.data()), "cf_item_graph_upload");
}

// "--name value" / "--name=value" option lookup.
inline std::string opt(int argc, char** argv, const std::string& name, const std::string& def) {
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--" + name && i + 1 < argc) return argv[i + 1];
        if (a.rfind("--" + name + "=", 0) == 0) return a.substr(name.size() + 3);
    }
    return def;
}

}  // namespace cfcli
