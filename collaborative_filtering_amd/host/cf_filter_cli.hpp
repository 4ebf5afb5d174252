// cf_filter_cli.hpp -- the file contract of cheby / binomials (cheby.cpp:296-380,
// binomials.cpp:255-367) around cf_graph_filter.
//   coeff*           every number, in file order (filter_loader, cheby.cpp:104-121)
//   graph_topology*  "va vb w" lines; w > 0.1 adds both directions (graph_loader, :88-92)
//   graph_signal*    "vt val" lines (graph_signal_loader, :94-102)
//   -> graph_filtered_signal_1_of_1: "id val" per vertex, ascending id, %g (graph_signal_writer,
//      :127-135; GraphLab's shard split and line order are unpinned upstream).
// A vertex that appears only in the topology has no signal line; the reference leaves its
// value uninitialised (vertex_data() { }), here it is 0.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "cf_cli.hpp"

namespace cffilt {

inline int run(int kind, const char* name) {
    std::vector<double> coeff;
    for (const auto& f : cfio::files_with_prefix(".", "coeff")) {
        const std::string text = cfio::read_file(f);
        const char* p = text.c_str();
        char* end = nullptr;
        for (;;) {
            const double v = std::strtod(p, &end);
            if (end == p) break;
            coeff.push_back(v);
            p = end;
        }
    }
    std::vector<uint32_t> la, lb;
    std::vector<double> lw;
    for (const auto& f : cfio::files_with_prefix(".", "graph_topology")) {
        const std::string text = cfio::read_file(f);
        const char* p = text.c_str();
        char* end = nullptr;
        for (;;) {
            const unsigned long a = std::strtoul(p, &end, 10);
            if (end == p) break;
            p = end;
            const unsigned long b = std::strtoul(p, &end, 10);
            if (end == p) break;
            p = end;
            const double w = std::strtod(p, &end);
            if (end == p) break;
            p = end;
            la.push_back((uint32_t)a);
            lb.push_back((uint32_t)b);
            lw.push_back(w);
        }
    }
    std::vector<std::pair<uint32_t, double>> sig;
    for (const auto& f : cfio::files_with_prefix(".", "graph_signal")) {
        const std::string text = cfio::read_file(f);
        const char* p = text.c_str();
        char* end = nullptr;
        for (;;) {
            const unsigned long v = std::strtoul(p, &end, 10);
            if (end == p) break;
            p = end;
            const double x = std::strtod(p, &end);
            if (end == p) break;
            p = end;
            sig.emplace_back((uint32_t)v, x);
        }
    }
    std::vector<uint32_t> all;
    for (size_t l = 0; l < lw.size(); ++l)
        if (lw[l] > 0.1) {   // only an added edge creates its vertices
            all.push_back(la[l]);
            all.push_back(lb[l]);
        }
    for (auto& s : sig) all.push_back(s.first);
    cfio::IdMap ids;
    ids.build(all);
    const uint32_t n = ids.size();
    std::vector<double> x(n, 0.0);
    for (auto& s : sig) x[ids.at[s.first]] = s.second;   // a repeated vertex: the last line wins
    std::vector<uint32_t> va, vb;
    std::vector<double> w;
    for (size_t l = 0; l < lw.size(); ++l) {
        if (!(lw[l] > 0.1)) continue;
        va.push_back(ids.at[la[l]]);
        vb.push_back(ids.at[lb[l]]);
        w.push_back(lw[l]);
    }
    std::fprintf(stderr, "%s: %u vertices, %zu topology lines kept, filter length %zu\n", name, n, w.size(),
                 coeff.size());
    cf_ctx* ctx = cfcli::open_device();
    std::vector<double> y(n);
    cfcli::check(ctx,
                 cf_graph_filter(ctx, kind, n, w.size(), va.data(), vb.data(), w.data(), x.data(), coeff.data(),
                                 (uint32_t)coeff.size(), y.data()),
                 "cf_graph_filter");
    float ms = 0.0f;
    uint64_t ne = 0;
    cf_graph_filter_timing(ctx, &ms, &ne);
    std::fprintf(stderr, "%s: %llu directed edges, device time %.3f ms\n", name, (unsigned long long)ne, ms);
    cf_destroy(ctx);
    cfio::ShardWriter out(".", "graph_filtered_signal", 1);
    for (uint32_t i = 0; i < n; ++i) {
        std::string& s = out.shard(ids.ids[i]);
        cfio::append_u(s, ids.ids[i]);
        s += ' ';
        cfio::append_g(s, y[i]);
        s += '\n';
    }
    out.flush();
    return 0;
}

}  // namespace cffilt
