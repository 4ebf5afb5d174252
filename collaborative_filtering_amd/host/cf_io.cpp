// cf_io.cpp -- text-file contract of the reference (see cf_io.hpp).
#include "cf_io.hpp"

#include <algorithm>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <thread>

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

namespace {

constexpr char kEigenMagic[8] = {'C', 'F', 'E', 'I', 'G', 'E', 'N', '1'};

// One 3-line text record (load_precomputed_data's state machine, local_calc_precomp.cpp:
// 426-476) from its three line spans; false on a malformed line (the reference asserts).
bool parse_eigen_record(const char* const* lb, const char* const* le, EigenRecord& cur) {
    uint32_t kk = 0, mm = 0;
    bool ok = true;
    {   // "uid k m" + "movie sig" x k (:426-442)
        Tok t{lb[0], le[0]};
        if (!t.u32(cur.user) || !t.u32(kk) || !t.u32(mm)) return false;
        cur.movies.resize(kk);
        cur.sigs.resize(kk);
        for (uint32_t i = 0; i < kk; ++i)
            if (!t.u32(cur.movies[i]) || !t.f64(cur.sigs[i])) ok = false;   // assert (:434)
    }
    {   // m eigenvalues (:444-452)
        Tok t{lb[1], le[1]};
        cur.evals.resize(mm);
        for (uint32_t i = 0; i < mm; ++i)
            if (!t.f64(cur.evals[i])) ok = false;   // assert (:447)
    }
    {   // k x m eigenvectors (:454-476)
        Tok t{lb[2], le[2]};
        cur.evecs.resize((size_t)kk * mm);
        for (size_t i = 0; i < (size_t)kk * mm; ++i)
            if (!t.f64(cur.evecs[i])) ok = false;   // assert (:462)
    }
    return ok;
}

int resolve_threads(int n_threads) {
    if (n_threads > 0) return n_threads;
    const unsigned h = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(h, 64u));
}

// Run f(t) for t in [0, n) on n threads (inline when n == 1).
template <class F>
void parallel_for(int n, F&& f) {
    if (n <= 1) {
        f(0);
        return;
    }
    std::vector<std::thread> pool;
    for (int t = 0; t < n; ++t) pool.emplace_back([&, t] { f(t); });
    for (auto& th : pool) th.join();
}

std::vector<EigenRecord> load_eigen_binary(const std::string& text, const std::string& path) {
    std::vector<EigenRecord> out;
    size_t pos = sizeof(kEigenMagic);
    auto take = [&](void* dst, size_t bytes) {
        if (pos + bytes > text.size()) throw std::runtime_error("truncated binary out_eigen_ " + path);
        std::memcpy(dst, text.data() + pos, bytes);
        pos += bytes;
    };
    uint64_t n = 0;
    take(&n, sizeof(n));
    out.resize(n);
    std::vector<float> buf;
    for (auto& r : out) {
        uint32_t hdr[3];
        take(hdr, sizeof(hdr));
        const uint32_t k = hdr[1], m = hdr[2];
        r.user = hdr[0];
        r.movies.resize(k);
        take(r.movies.data(), sizeof(uint32_t) * k);
        auto floats = [&](std::vector<double>& dst, size_t cnt) {
            buf.resize(cnt);
            take(buf.data(), sizeof(float) * cnt);
            dst.assign(buf.begin(), buf.end());
        };
        floats(r.sigs, k);
        floats(r.evals, m);
        floats(r.evecs, (size_t)k * m);
    }
    return out;
}

}  // namespace

std::vector<EigenRecord> load_eigen_file(const std::string& path, int n_threads) {
    const std::string text = read_file(path);
    if (text.size() >= sizeof(kEigenMagic) && std::memcmp(text.data(), kEigenMagic, sizeof(kEigenMagic)) == 0)
        return load_eigen_binary(text, path);
    // non-empty line spans, then records of 3 lines parsed in parallel over record ranges
    std::vector<const char*> lb, le;
    {
        const char* p = text.data();
        const char* end = p + text.size();
        while (p < end) {
            const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
            if (!nl) nl = end;
            if (nl > p) {
                lb.push_back(p);
                le.push_back(nl);
            }
            p = nl + 1;
        }
    }
    const size_t n_rec = lb.size() / 3;   // a trailing partial record is dropped (state machine)
    std::vector<EigenRecord> out(n_rec);
    const int T = (int)std::min<size_t>((size_t)resolve_threads(n_threads), std::max<size_t>(n_rec, 1));
    std::vector<char> bad(T, 0);
    parallel_for(T, [&](int t) {
        const size_t r0 = n_rec * t / T, r1 = n_rec * (t + 1) / T;
        for (size_t r = r0; r < r1; ++r)
            if (!parse_eigen_record(&lb[3 * r], &le[3 * r], out[r])) bad[t] = 1;
    });
    for (char b : bad)
        if (b) throw std::runtime_error("malformed out_eigen_ record in " + path);
    return out;
}

void write_eigen_file(const std::string& path, bool append, int n_threads, bool binary, uint32_t n_users,
                      const uint32_t* uid, const uint64_t* off, const int32_t* m, const uint32_t* movies,
                      const float* sigs, const float* evals, const uint64_t* eoff, const float* evecs) {
    std::ofstream f(path, std::ofstream::binary | (append ? std::ofstream::app : std::ofstream::trunc));
    if (!f) throw std::runtime_error("cannot open " + path);
    if (binary) {   // "CFEIGEN1", n, then per record uid k m movies[k] sigs[k] evals[m] evecs[k*m]
        const uint64_t n = n_users;
        f.write(kEigenMagic, sizeof(kEigenMagic));
        f.write(reinterpret_cast<const char*>(&n), sizeof(n));
        std::vector<float> ev;
        for (uint32_t u = 0; u < n_users; ++u) {
            const uint32_t k = (uint32_t)(off[u + 1] - off[u]), mm = (uint32_t)m[u];
            const uint32_t hdr[3] = {uid[u], k, mm};
            f.write(reinterpret_cast<const char*>(hdr), sizeof(hdr));
            f.write(reinterpret_cast<const char*>(movies + off[u]), sizeof(uint32_t) * k);
            f.write(reinterpret_cast<const char*>(sigs + off[u]), sizeof(float) * k);
            ev.assign(mm, 0.0f);   // entries past k (k == 1 padding) are 0, as in the text form
            for (uint32_t j = 0; j < mm && j < k; ++j) ev[j] = evals[off[u] + j];
            f.write(reinterpret_cast<const char*>(ev.data()), sizeof(float) * mm);
            f.write(reinterpret_cast<const char*>(evecs + eoff[u]), sizeof(float) * (size_t)k * mm);
        }
        return;
    }
    // text: contiguous user ranges formatted in parallel, written in order
    const int T = (int)std::min<uint32_t>((uint32_t)resolve_threads(n_threads), std::max<uint32_t>(n_users, 1));
    const uint32_t chunk = 4096;   // users per formatting task
    const uint32_t n_chunks = (n_users + chunk - 1) / chunk;
    for (uint32_t c0 = 0; c0 < n_chunks; c0 += (uint32_t)T) {
        const int nt = (int)std::min<uint32_t>((uint32_t)T, n_chunks - c0);
        std::vector<std::string> part(nt);
        parallel_for(nt, [&](int t) {
            const uint32_t u0 = (c0 + t) * chunk, u1 = std::min(n_users, u0 + chunk);
            for (uint32_t u = u0; u < u1; ++u) {
                const uint32_t k = (uint32_t)(off[u + 1] - off[u]);
                append_eigen_record(part[t], uid[u], k, (uint32_t)m[u], movies + off[u], sigs + off[u],
                                    evals + off[u], evecs + eoff[u]);
            }
        });
        for (auto& p : part) f.write(p.data(), (std::streamsize)p.size());
    }
}

}  // namespace cfio

// C entry points used by the Python side (tests compare the formatting with printf, and the
// parallel / binary out_eigen_ writers and readers with the serial text form).
extern "C" int cfh_write_eigen(const char* path, int append, int n_threads, int binary, uint32_t n_users,
                               const uint32_t* uid, const uint64_t* off, const int32_t* m, const uint32_t* movies,
                               const float* sigs, const float* evals, const uint64_t* eoff, const float* evecs) {
    try {
        cfio::write_eigen_file(path, append != 0, n_threads, binary != 0, n_users, uid, off, m, movies, sigs, evals,
                               eoff, evecs);
    } catch (const std::exception&) {
        return -1;
    }
    return 0;
}

// Loads out_eigen_ (text or binary) and returns the record count; when `flat` is non-null it
// receives, per record, uid, k, m, then movies, sigs, evals, evecs as doubles (cap doubles).
extern "C" int64_t cfh_load_eigen(const char* path, int n_threads, double* flat, int64_t cap) {
    try {
        const auto recs = cfio::load_eigen_file(path, n_threads);
        int64_t pos = 0;
        auto put = [&](double v) {
            if (flat && pos < cap) flat[pos] = v;
            ++pos;
        };
        for (const auto& r : recs) {
            put(r.user);
            put((double)r.movies.size());
            put((double)r.evals.size());
            for (auto v : r.movies) put(v);
            for (auto v : r.sigs) put(v);
            for (auto v : r.evals) put(v);
            for (auto v : r.evecs) put(v);
        }
        if (flat && pos > cap) return -2;
        return (int64_t)recs.size();
    } catch (const std::exception&) {
        return -1;
    }
}

// C entry points used by the Python side (tests compare the formatting with printf).
extern "C" int cfh_format_g(double v, char* buf, int cap) {
    std::string s;
    cfio::append_g(s, v);
    if ((int)s.size() + 1 > cap) return -1;
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return (int)s.size();
}
