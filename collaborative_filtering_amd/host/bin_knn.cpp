// knn -- drop-in for knn.cpp (a9): regroup movielens/ ratings into per-movie train
// (out_rat_), test (out_test_rat_) and co-rated movie lists (out_edg_).
//   knn.cpp:83-111  loader: role by file suffix, user id -> uimax - id
//   knn.cpp:160-205 engine 1: movie gathers IN_EDGES -> ratings / ratings_test
//   knn.cpp:212-298 engines 2-3: co-rated movie set per movie (train AND validate)
//   knn.cpp:303-357 writers (movie vertices only; sorted unique, self removed)
#include <algorithm>
#include <cstdio>
#include <map>

#include "cf_cli.hpp"

int main(int argc, char** argv) {
    const std::string dir = cfcli::opt(argc, argv, "input", "movielens/");
    const int nshards = std::stoi(cfcli::opt(argc, argv, "nshards", "4"));
    std::vector<cfio::Rating> rs = cfio::load_movielens(dir, true);
    std::printf("Loaded %zu ratings from %s\n", rs.size(), dir.c_str());
    // map semantics: per (movie, user) the last rating read wins, per role
    std::map<uint32_t, std::map<uint32_t, double>> train, test;
    std::map<uint32_t, std::vector<uint32_t>> user_movies;
    for (const auto& r : rs) {
        (r.validate ? test : train)[r.movie][r.user] = r.value;
        if (!r.validate) test[r.movie];   // movie vertex exists either way
        else train[r.movie];
        user_movies[r.user].push_back(r.movie);
    }
    std::vector<uint32_t> movies;
    for (auto& kv : train) movies.push_back(kv.first);
    cfio::IdMap ids;
    ids.build(movies);
    // co-rated sets: union over the movie's raters of their movies (both roles, :224-227,271-274)
    std::vector<std::vector<uint32_t>> corated(ids.size());
    for (auto& kv : user_movies) {
        auto& ms = kv.second;
        std::sort(ms.begin(), ms.end());
        ms.erase(std::unique(ms.begin(), ms.end()), ms.end());
        for (uint32_t a : ms)
            for (uint32_t b : ms)
                if (a != b) corated[ids.at[a]].push_back(b);
    }
    cfio::ShardWriter rat(".", "out_rat", nshards), trat(".", "out_test_rat", nshards), edg(".", "out_edg", nshards);
    for (uint32_t i = 0; i < ids.size(); ++i) {
        const uint32_t m = ids.ids[i];
        for (int which = 0; which < 2; ++which) {
            std::string& out = which ? trat.shard(m) : rat.shard(m);
            cfio::append_u(out, m);
            out += ' ';
            for (auto& ur : (which ? test : train)[m]) {   // :307-309, :324-326
                cfio::append_u(out, ur.first);
                out += ' ';
                cfio::append_g(out, ur.second);
                out += ' ';
            }
            out += '\n';
        }
        auto& c = corated[i];
        std::sort(c.begin(), c.end());
        c.erase(std::unique(c.begin(), c.end()), c.end());
        std::string& out = edg.shard(m);
        cfio::append_u(out, m);
        out += ' ';
        for (uint32_t b : c) {   // :342-351
            cfio::append_u(out, b);
            out += ' ';
        }
        out += '\n';
    }
    rat.flush();
    trat.flush();
    edg.flush();
    std::printf("Wrote out_rat_, out_test_rat_, out_edg_ for %u movies\n", ids.size());
    return 0;
}
