// cf_io.cpp -- text-file contract of the reference (see cf_io.hpp).
#include "cf_io.hpp"

#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace cfio {

namespace {

bool ends_with(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}
bool starts_with(const std::string& s, const std::string& pre) { return s.compare(0, pre.size(), pre) == 0; }

std::vector<std::string> list_dir(const std::string& dir) {
    std::vector<std::string> out;
    DIR* d = opendir(dir.empty() ? "." : dir.c_str());
    if (!d) return out;
    while (dirent* e = readdir(d)) {
        std::string name = e->d_name;
        if (name == "." || name == "..") continue;
        const std::string full = (dir.empty() ? std::string() : (ends_with(dir, "/") ? dir : dir + "/")) + name;
        struct stat st;
        if (stat(full.c_str(), &st) == 0 && S_ISREG(st.st_mode)) out.push_back(name);
    }
    closedir(d);
    std::sort(out.begin(), out.end());
    return out;
}

std::string join(const std::string& dir, const std::string& name) {
    if (dir.empty() || dir == ".") return name;
    return ends_with(dir, "/") ? dir + name : dir + "/" + name;
}

// Tokenizer over one line.
struct Tok {
    const char* p;
    const char* e;
    void skip() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
    }
    bool u32(uint32_t& v) {
        skip();
        auto r = std::from_chars(p, e, v);
        if (r.ec != std::errc()) return false;
        p = r.ptr;
        return true;
    }
    bool f64(double& v) {
        skip();
        if (p < e && *p == '+') ++p;
        auto r = std::from_chars(p, e, v);
        if (r.ec != std::errc()) return false;
        p = r.ptr;
        return true;
    }
};

template <typename F>
void for_each_line(const std::string& text, F&& f) {
    size_t pos = 0;
    while (pos < text.size()) {
        size_t nl = text.find('\n', pos);
        if (nl == std::string::npos) nl = text.size();
        if (nl > pos) f(text.data() + pos, text.data() + nl);
        pos = nl + 1;
    }
}

}  // namespace

std::vector<std::string> files_with_suffix(const std::string& dir, const std::string& suffix) {
    std::vector<std::string> out;
    for (auto& n : list_dir(dir))
        if (suffix.empty() || ends_with(n, suffix)) out.push_back(join(dir, n));
    return out;
}

std::vector<std::string> files_with_prefix(const std::string& dir, const std::string& prefix) {
    std::vector<std::string> out;
    for (auto& n : list_dir(dir))
        if (prefix.empty() || starts_with(n, prefix)) out.push_back(join(dir, n));
    return out;
}

std::string read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::ostringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

void append_g(std::string& out, double v) {
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::general, 6);
    out.append(buf, r.ptr);
}

void append_u(std::string& out, uint64_t v) {
    char buf[32];
    auto r = std::to_chars(buf, buf + sizeof(buf), v);
    out.append(buf, r.ptr);
}

std::vector<Rating> load_movielens(const std::string& dir, bool remap_users) {
    std::vector<Rating> out;
    for (const auto& path : files_with_suffix(dir, "")) {
        const bool validate = ends_with(path, ".validate");
        const std::string text = read_file(path);
        for_each_line(text, [&](const char* b, const char* e) {
            Tok t{b, e};
            uint32_t u, m;
            double r = 0;
            if (!t.u32(u) || !t.u32(m)) return;
            t.f64(r);  // .predict lines carry no rating (read as 0, knn.cpp:97-98)
            out.push_back({remap_users ? kUimax - u : u, m, r, validate});
        });
    }
    return out;
}

VertexRatings load_vertex_ratings(const std::string& dir, const std::string& prefix, bool require_nonempty) {
    VertexRatings out;
    for (const auto& path : files_with_prefix(dir, prefix)) {
        const std::string text = read_file(path);
        for_each_line(text, [&](const char* b, const char* e) {
            Tok t{b, e};
            uint32_t vt;
            if (!t.u32(vt)) return;
            std::vector<std::pair<uint32_t, double>> rs;
            uint32_t u;
            double r;
            while (t.u32(u) && t.f64(r)) rs.push_back({u, r});
            if (require_nonempty && rs.empty()) return;   // graph_test_loader (:156-157)
            auto& dst = out[vt];
            dst.insert(dst.end(), rs.begin(), rs.end());
        });
    }
    // map semantics: one rating per (vertex, user), the last one read wins
    for (auto& kv : out) {
        auto& v = kv.second;
        std::stable_sort(v.begin(), v.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        size_t w = 0;
        for (size_t i = 0; i < v.size(); ++i) {
            if (w > 0 && v[w - 1].first == v[i].first)
                v[w - 1] = v[i];
            else
                v[w++] = v[i];
        }
        v.resize(w);
    }
    return out;
}

std::vector<Edge> load_edges(const std::string& dir, const std::string& prefix) {
    std::vector<Edge> out;
    for (const auto& path : files_with_prefix(dir, prefix)) {
        const std::string text = read_file(path);
        for_each_line(text, [&](const char* b, const char* e) {
            Tok t{b, e};
            uint32_t a, c;
            double w;
            if (t.u32(a) && t.u32(c) && t.f64(w)) out.push_back({a, c, w});
        });
    }
    return out;
}

std::vector<std::pair<uint32_t, uint32_t>> load_adjacency(const std::string& dir, const std::string& prefix) {
    std::vector<std::pair<uint32_t, uint32_t>> out;
    for (const auto& path : files_with_prefix(dir, prefix)) {
        const std::string text = read_file(path);
        for_each_line(text, [&](const char* b, const char* e) {
            Tok t{b, e};
            uint32_t a, c;
            if (!t.u32(a)) return;
            while (t.u32(c)) out.push_back({a, c});
        });
    }
    return out;
}

ShardWriter::ShardWriter(const std::string& dir, const std::string& prefix, int nshards)
    : dir_(dir), prefix_(prefix), buf_(std::max(1, nshards)) {}

void ShardWriter::flush() {
    const int n = (int)buf_.size();
    for (int i = 0; i < n; ++i) {
        const std::string path = join(dir_, prefix_ + "_" + std::to_string(i + 1) + "_of_" + std::to_string(n));
        std::ofstream f(path, std::ios::binary | std::ios::trunc);
        if (!f) throw std::runtime_error("cannot write " + path);
        f.write(buf_[i].data(), (std::streamsize)buf_[i].size());
        buf_[i].clear();
    }
}

void IdMap::build(std::vector<uint32_t> all) {
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
    ids = std::move(all);
    at.clear();
    at.reserve(ids.size() * 2);
    for (uint32_t i = 0; i < ids.size(); ++i) at[ids[i]] = i;
}

void append_eigen_record(std::string& out, uint32_t user, uint32_t k, uint32_t m, const uint32_t* movies,
                         const float* sigs, const float* evals, const float* evecs) {
    // line 1: "uid k m " + "movie sig " x k   (:197-199)
    append_u(out, user);
    out += ' ';
    append_u(out, k);
    out += ' ';
    append_u(out, m);
    out += ' ';
    for (uint32_t i = 0; i < k; ++i) {
        append_u(out, movies[i]);
        out += ' ';
        append_g(out, (double)sigs[i]);
        out += ' ';
    }
    out += '\n';
    // line 2: m eigenvalues (:201-203); entries past k (k == 1 padding) are 0
    for (uint32_t j = 0; j < m; ++j) {
        append_g(out, j < k ? (double)evals[j] : 0.0);
        out += ' ';
    }
    out += '\n';
    // line 3: k x m eigenvectors row-major (:205-209)
    for (uint64_t t = 0; t < (uint64_t)k * m; ++t) {
        append_g(out, (double)evecs[t]);
        out += ' ';
    }
    out += '\n';
}

std::vector<EigenRecord> load_eigen_file(const std::string& path) {
    std::vector<EigenRecord> out;
    const std::string text = read_file(path);
    int state = 0;
    EigenRecord cur;
    uint32_t kk = 0, mm = 0;
    bool bad = false;
    for_each_line(text, [&](const char* b, const char* e) {
        Tok t{b, e};
        switch (state) {
            case 0: {  // (:426-442)
                cur = EigenRecord();
                if (!t.u32(cur.user) || !t.u32(kk) || !t.u32(mm)) {
                    bad = true;
                    return;
                }
                cur.movies.resize(kk);
                cur.sigs.resize(kk);
                for (uint32_t i = 0; i < kk; ++i)
                    if (!t.u32(cur.movies[i]) || !t.f64(cur.sigs[i])) bad = true;  // assert (:434)
                state = 1;
                break;
            }
            case 1:  // (:444-452)
                cur.evals.resize(mm);
                for (uint32_t i = 0; i < mm; ++i)
                    if (!t.f64(cur.evals[i])) bad = true;  // assert (:447)
                state = 2;
                break;
            case 2:  // (:454-476)
                cur.evecs.resize((size_t)kk * mm);
                for (size_t i = 0; i < (size_t)kk * mm; ++i)
                    if (!t.f64(cur.evecs[i])) bad = true;  // assert (:462)
                out.push_back(std::move(cur));
                state = 0;
                break;
        }
    });
    if (bad) throw std::runtime_error("malformed out_eigen_ record in " + path);
    return out;
}

}  // namespace cfio

// C entry points used by the Python side (tests compare the formatting with printf).
extern "C" int cfh_format_g(double v, char* buf, int cap) {
    std::string s;
    cfio::append_g(s, v);
    if ((int)s.size() + 1 > cap) return -1;
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return (int)s.size();
}
