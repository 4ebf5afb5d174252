// knn -- drop-in for knn.cpp (a9): regroup movielens/ ratings into per-movie train
// (out_rat_), test (out_test_rat_) and co-rated movie lists (out_edg_).
//   knn.cpp:83-111  loader: role by file suffix, user id -> uimax - id
//   knn.cpp:160-205 engine 1: movie gathers IN_EDGES -> ratings / ratings_test
//   knn.cpp:212-298 engines 2-3: co-rated movie set per movie (train AND validate)
//   knn.cpp:303-357 writers (movie vertices only; sorted unique, self removed)
// The grouping (last rating per (role, movie, user), per-movie lists, co-rated sets) runs on
// the GPU (cf_knn_regroup); this file parses and formats.
#include <algorithm>
#include <cstdio>
#include <unordered_map>

#include "cf_cli.hpp"

int main(int argc, char** argv) {
    const std::string dir = cfcli::opt(argc, argv, "input", "movielens/");
    const int nshards = std::stoi(cfcli::opt(argc, argv, "nshards", "4"));
    std::vector<cfio::Rating> rs = cfio::load_movielens(dir, true);
    std::printf("Loaded %zu ratings from %s\n", rs.size(), dir.c_str());
    // compact ids: users in remapped-id order (the maps' iteration order), movies ascending
    std::vector<uint32_t> all_u, all_m;
    for (const auto& r : rs) {
        all_u.push_back(r.user);
        all_m.push_back(r.movie);
    }
    cfio::IdMap uids, ids;
    uids.build(all_u);
    ids.build(all_m);
    const uint64_t n = rs.size();
    std::vector<uint32_t> cu(n), cm(n);
    std::vector<float> fr(n);
    std::vector<uint8_t> role(n);
    // the printed value is the parsed double of the rating that wins (the last one read per
    // (role, movie, user), map assignment); the GPU groups by compact ids
    std::unordered_map<uint64_t, double> value;
    value.reserve(n * 2);
    for (uint64_t i = 0; i < n; ++i) {
        cu[i] = uids.at[rs[i].user];
        cm[i] = ids.at[rs[i].movie];
        fr[i] = (float)rs[i].value;
        role[i] = rs[i].validate;
        value[((uint64_t)(role[i] * ids.size() + cm[i]) << 32) | cu[i]] = rs[i].value;
    }
    const uint32_t nm = ids.size();
    std::vector<uint64_t> tro(nm + 1), teo(nm + 1), eo(nm + 1);
    std::vector<uint32_t> tru(n), teu(n);
    std::vector<float> trr(n), ter(n);
    std::vector<uint32_t> edg;
    cf_ctx* ctx = cfcli::open_device();
    uint64_t cap = std::min<uint64_t>((uint64_t)nm * (nm > 0 ? nm - 1 : 0), 1ull << 26);
    for (;;) {   // co-rated lists beyond the first guess: retry with the exact size
        edg.resize(cap);
        const int rc = cf_knn_regroup(ctx, n, uids.size(), nm, cu.data(), cm.data(), fr.data(), role.data(),
                                      tro.data(), tru.data(), trr.data(), teo.data(), teu.data(), ter.data(),
                                      eo.data(), edg.data(), cap);
        if (rc == CF_ERANGE && eo[nm] > cap) {
            cap = eo[nm];
            continue;
        }
        cfcli::check(ctx, rc, "cf_knn_regroup");
        break;
    }
    cf_destroy(ctx);
    cfio::ShardWriter rat(".", "out_rat", nshards), trat(".", "out_test_rat", nshards), edg_out(".", "out_edg", nshards);
    for (uint32_t i = 0; i < nm; ++i) {
        const uint32_t m = ids.ids[i];
        for (int which = 0; which < 2; ++which) {
            std::string& out = which ? trat.shard(m) : rat.shard(m);
            const uint64_t* off = which ? teo.data() : tro.data();
            const uint32_t* us = which ? teu.data() : tru.data();
            cfio::append_u(out, m);
            out += ' ';
            for (uint64_t j = off[i]; j < off[i + 1]; ++j) {   // :307-309, :324-326
                cfio::append_u(out, uids.ids[us[j]]);
                out += ' ';
                cfio::append_g(out, value.at(((uint64_t)(which * nm + i) << 32) | us[j]));
                out += ' ';
            }
            out += '\n';
        }
        std::string& out = edg_out.shard(m);
        cfio::append_u(out, m);
        out += ' ';
        for (uint64_t j = eo[i]; j < eo[i + 1]; ++j) {   // :342-351
            cfio::append_u(out, ids.ids[edg[j]]);
            out += ' ';
        }
        out += '\n';
    }
    rat.flush();
    trat.flush();
    edg_out.flush();
    std::printf("Wrote out_rat_, out_test_rat_, out_edg_ for %u movies\n", nm);
    return 0;
}
