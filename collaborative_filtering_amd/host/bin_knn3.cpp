// knn3 -- drop-in for knn3.cpp (a11): weighted-average kNN prediction over the
// out_fin_ edges with w > 0.1 and the test ratings of out_test_rat_; prints
// "Knn Average MSE: <sum of per-vertex MSE / num_vertices>" (knn3.cpp:261-264).
#include <cmath>
#include <cstdio>

#include "cf_cli.hpp"

int main(int, char**) {
    auto edges = cfio::load_edges(".", "out_fin_");
    cfio::VertexRatings test = cfio::load_vertex_ratings(".", "out_test_rat_", true);   // :97-119
    std::vector<uint32_t> all, verts;
    for (auto& e : edges) {
        all.push_back(e.a);
        all.push_back(e.b);
        if ((float)e.w > 0.1) {   // graph_loader: float weight > 0.1 creates the edge (:88-92)
            verts.push_back(e.a);
            verts.push_back(e.b);
        }
    }
    for (auto& kv : test) {
        all.push_back(kv.first);
        verts.push_back(kv.first);
    }
    cfio::IdMap items, vset;
    items.build(all);
    vset.build(verts);
    // out_fin_ weights as parsed floats; the kernel applies the > 0.1 threshold
    std::vector<cfio::Edge> fe = edges;
    for (auto& e : fe) e.w = (double)(float)e.w;
    cf_ctx* ctx = cfcli::open_device();
    cfcli::upload_edges(ctx, items, fe);
    // regroup test ratings by user
    std::vector<uint32_t> uids;
    for (auto& kv : test)
        for (auto& ur : kv.second) uids.push_back(ur.first);
    cfio::IdMap users;
    users.build(uids);
    std::vector<uint64_t> off(users.size() + 1, 0);
    for (auto& kv : test)
        for (auto& ur : kv.second) off[users.at[ur.first] + 1]++;
    for (uint32_t u = 0; u < users.size(); ++u) off[u + 1] += off[u];
    std::vector<uint32_t> it(off.back());
    std::vector<float> r(off.back());
    std::vector<uint64_t> fill(off.begin(), off.end() - 1);
    for (auto& kv : test)
        for (auto& ur : kv.second) {
            const uint64_t p = fill[users.at[ur.first]]++;
            it[p] = items.at[kv.first];
            r[p] = (float)ur.second;
        }
    std::vector<float> mse(items.size());
    cfcli::check(ctx, cf_knn_predict(ctx, users.size(), off.data(), it.data(), r.data(), nullptr, mse.data(), nullptr),
                 "cf_knn_predict");
    cf_destroy(ctx);
    float total = 0.0f;   // aggregator sum (:324-327), ascending vertex id
    for (uint32_t i = 0; i < items.size(); ++i) total += mse[i];
    const float avg = total / (float)vset.size();
    std::string line = "Knn Average MSE: ";
    cfio::append_g(line, (double)avg);
    std::printf("%s\n", line.c_str());
    return 0;
}
