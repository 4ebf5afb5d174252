// knn2 -- drop-in for knn2.cpp (a10): cosine item weights on the out_edg_ edges from
// the out_rat_ train maps; writes out_fin_ "a b w" for w > 0.01 (knn2.cpp:151-164).
// Optional --topk K (off by default): only the K largest weights per source item.
// The weights come from cf_item_cosine_edges (int8 / fp32 MFMA over all item pairs, compacted
// on the device to the w > 0.01 edge list); the writer keeps exactly the out_edg_ edges, in
// out_edg_ order per source.
#include <algorithm>
#include <cstdio>

#include "cf_cli.hpp"

int main(int argc, char** argv) {
    const int nshards = std::stoi(cfcli::opt(argc, argv, "nshards", "4"));
    // --topk K (default 0 = off, the reference's threshold-only neighbourhoods): keep the K
    // largest weights per source item (ties: lower item ids), cf_set_knn2_topk
    const long topk = std::stol(cfcli::opt(argc, argv, "topk", "0"));
    if (topk < 0) {
        std::fprintf(stderr, "knn2: --topk must be >= 0\n");
        return 2;
    }
    cfio::VertexRatings rat = cfio::load_vertex_ratings(".", "out_rat_", false);   // :79-102
    auto edges = cfio::load_adjacency(".", "out_edg_");                            // :104-121
    std::vector<uint32_t> all;
    for (auto& kv : rat) all.push_back(kv.first);
    for (auto& e : edges) {
        all.push_back(e.first);
        all.push_back(e.second);
    }
    cfio::IdMap items;
    items.build(all);
    // per-user train CSR over compact items
    std::vector<uint32_t> uids;
    for (auto& kv : rat)
        for (auto& ur : kv.second) uids.push_back(ur.first);
    cfio::IdMap users;
    users.build(uids);
    std::vector<uint64_t> off(users.size() + 1, 0);
    for (auto& kv : rat)
        for (auto& ur : kv.second) off[users.at[ur.first] + 1]++;
    for (uint32_t u = 0; u < users.size(); ++u) off[u + 1] += off[u];
    std::vector<uint32_t> it(off.back());
    std::vector<float> r(off.back());
    std::vector<uint64_t> fill(off.begin(), off.end() - 1);
    for (auto& kv : rat)
        for (auto& ur : kv.second) {
            const uint64_t p = fill[users.at[ur.first]]++;
            it[p] = items.at[kv.first];
            r[p] = (float)ur.second;
        }
    const uint32_t n = items.size();
    // knn2 as the compacted edge list (cf_item_cosine_edges): the dense similarity matrix is
    // compacted on the device, only the w > 0.01 edges come back (targets ascending per source)
    std::vector<uint64_t> eoff((size_t)n + 1);
    std::vector<uint32_t> ecol;
    std::vector<float> ew;
    uint64_t n_edges = 0;
    cf_ctx* ctx = cfcli::open_device();
    cfcli::check(ctx, cf_set_knn2_topk(ctx, (uint32_t)topk), "cf_set_knn2_topk");
    // Capacity: every w > 0.01 pair has cnt > 5 co-raters, so it is a co-rated pair and
    // out_edg_ (written by knn from the same ratings) lists it -- one call computes knn2.
    // Files from different runs can break that bound: the call then reports the size it
    // needs (CF_ERANGE) and runs once more.
    ecol.resize(edges.size());
    ew.resize(edges.size());
    int rc = cf_item_cosine_edges(ctx, users.size(), n, off.data(), it.data(), r.data(), 0.01f, 5, 0, eoff.data(),
                                  ecol.data(), ew.data(), ecol.size(), &n_edges);
    if (rc == CF_ERANGE && n_edges > ecol.size()) {
        ecol.resize(n_edges);
        ew.resize(n_edges);
        rc = cf_item_cosine_edges(ctx, users.size(), n, off.data(), it.data(), r.data(), 0.01f, 5, 0, eoff.data(),
                                  ecol.data(), ew.data(), n_edges, &n_edges);
    }
    cfcli::check(ctx, rc, "cf_item_cosine_edges");
    {
        double acc = 0.0;
        int exact = 0, path = 0;
        float pa = 0.0f, pb = 0.0f;
        cfcli::check(ctx, cf_knn2_exactness(ctx, &acc, &exact), "cf_knn2_exactness");
        cfcli::check(ctx, cf_knn2_timing(ctx, &pa, &pb, &path), "cf_knn2_timing");
        if (!exact && path != 3)
            std::fprintf(stderr,
                         "knn2: warning: an accumulator reaches %.0f > 2^24; the reference's float sums "
                         "(knn2.cpp:129-140) are no longer exact there, these weights are the exact ones\n",
                         acc);
    }
    cf_destroy(ctx);
    // w(a, b) of an out_edg_ pair: a binary search of a's edge list (0 when absent)
    const auto weight = [&](uint32_t a, uint32_t b) -> float {
        const uint32_t* lo = ecol.data() + eoff[a];
        const uint32_t* hi = ecol.data() + eoff[a + 1];
        const uint32_t* p = std::lower_bound(lo, hi, b);
        return (p != hi && *p == b) ? ew[(size_t)(p - ecol.data())] : 0.0f;
    };
    cfio::ShardWriter fin(".", "out_fin", nshards);
    size_t written = 0;
    for (auto& e : edges) {
        const float w = weight(items.at[e.first], items.at[e.second]);
        if (!(w > 0.0f)) continue;
        std::string& out = fin.shard(e.first);
        cfio::append_u(out, e.first);
        out += ' ';
        cfio::append_u(out, e.second);
        out += ' ';
        cfio::append_g(out, (double)w);
        out += '\n';
        ++written;
    }
    fin.flush();
    std::printf("Wrote %zu out_fin_ edges of %zu out_edg_ edges\n", written, edges.size());
    return 0;
}
