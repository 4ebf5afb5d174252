// cf_io.cpp -- text-file contract of the reference (see cf_io.hpp).
#include "cf_io.hpp"

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <thread>

#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

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

}  // namespace

bool parse_f64(const char*& p, const char* e, double& out);

namespace {

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
        return parse_f64(p, e, v);
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

// %g, precision 6.  Fast path for values exactly representable as float with 1e-3 <= |v| < 1e6
// (every eigenvector entry, eigenvalue, sig and mse the writers format, bar the tiny ones): with
// a 24-bit mantissa, n = |v| * 10^k (k <= 8, 10^k < 2^27) is EXACT in double, so nearbyint(n)
// is the correctly rounded 6-digit significand with ties to even -- printf's and to_chars'
// rounding of the exact binary value -- and the digits follow without any conversion error.
// Everything else takes std::to_chars (tests/test_formats.py compares both on millions of
// values, ties included).
char* format_g6(char* p, double v) {
    static const double kPow[9] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8};
    const double a = std::fabs(v);
    if (!(a >= 1e-3 && a < 1e6) || (double)(float)v != v)
        return std::to_chars(p, p + 32, v, std::chars_format::general, 6).ptr;
    int k = 0;
    double n = a;
    while (n < 1e5) n = a * kPow[++k];      // n in [1e5, 1e6), exact
    double r = std::nearbyint(n);            // round half even
    int x = 5 - k;                           // decimal exponent of the leading digit
    if (r >= 1e6) {                          // 999999.5 -> 1000000: one more digit position
        r = 1e5;
        if (++x >= 6) return std::to_chars(p, p + 32, v, std::chars_format::general, 6).ptr;
    }
    uint32_t d = (uint32_t)r;
    char dig[6];
    for (int i = 5; i >= 0; --i) {
        dig[i] = (char)('0' + d % 10);
        d /= 10;
    }
    int nd = 6;                              // significant digits left after stripping zeros
    while (nd > x + 1 && nd > 1 && dig[nd - 1] == '0') --nd;
    if (v < 0) *p++ = '-';
    if (x >= 0) {                            // ddd.ddd
        for (int i = 0; i <= x; ++i) *p++ = dig[i];
        if (nd > x + 1) {
            *p++ = '.';
            for (int i = x + 1; i < nd; ++i) *p++ = dig[i];
        }
    } else {                                 // 0.000ddd
        *p++ = '0';
        *p++ = '.';
        for (int i = 0; i < -x - 1; ++i) *p++ = '0';
        for (int i = 0; i < nd; ++i) *p++ = dig[i];
    }
    return p;
}

void append_g(std::string& out, double v) {
    char buf[64];
    out.append(buf, format_g6(buf, v));
}

// strtod-exact parse of a decimal number: Clinger's fast path (mantissa < 2^53 and a power of
// ten up to 10^22 are exact doubles, so one multiplication or division is correctly rounded)
// for the short numbers of these files, std::from_chars otherwise.  Accepts what from_chars
// accepts plus a leading '+'.
bool parse_f64(const char*& p, const char* e, double& out) {
    static const double kPow[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                    1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    const char* q = p;
    if (q < e && *q == '+') ++q;
    const char* start = q;
    bool neg = false;
    if (q < e && *q == '-') {
        neg = true;
        ++q;
    }
    uint64_t w = 0;
    int nd = 0, ex = 0;
    bool any = false;
    while (q < e && (unsigned)(*q - '0') < 10) {
        if (nd < 19) w = w * 10 + (uint64_t)(*q - '0'), nd += (w != 0);
        else ++ex;
        ++q;
        any = true;
    }
    if (q < e && *q == '.') {
        ++q;
        while (q < e && (unsigned)(*q - '0') < 10) {
            if (nd < 19) {
                w = w * 10 + (uint64_t)(*q - '0');
                nd += (w != 0);
                --ex;
            }
            ++q;
            any = true;
        }
    }
    if (q < e && (*q == 'e' || *q == 'E')) {
        const char* t = q + 1;
        bool eneg = false;
        if (t < e && (*t == '+' || *t == '-')) eneg = *t++ == '-';
        int ev = 0;
        bool edig = false;
        while (t < e && (unsigned)(*t - '0') < 10 && ev < 10000) ev = ev * 10 + (*t++ - '0'), edig = true;
        if (edig) {
            ex += eneg ? -ev : ev;
            q = t;
        }
    }
    if (any && nd < 19 && w < (1ull << 53) && ex >= -22 && ex <= 22 && (q == e || (unsigned)(*q - '0') >= 10)) {
        double d = (double)w;
        d = ex < 0 ? d / kPow[-ex] : d * kPow[ex];
        out = neg ? -d : d;
        p = q;
        return true;
    }
    auto r = std::from_chars(start, e, out);
    if (r.ec != std::errc()) return false;
    p = r.ptr;
    return true;
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

// Read-only mapping of a whole file (empty files map to nothing).
struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    // populate: fault the whole file in at map time (one kernel thread); otherwise the parsing
    // threads fault their own ranges in parallel
    explicit Mapped(const std::string& path, bool populate = true) {
        const int fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) throw std::runtime_error("cannot open " + path);
        struct stat st;
        if (fstat(fd, &st) != 0) {
            ::close(fd);
            throw std::runtime_error("cannot stat " + path);
        }
        n = (size_t)st.st_size;
        if (n) {
            void* v = mmap(nullptr, n, PROT_READ, MAP_PRIVATE | (populate ? MAP_POPULATE : 0), fd, 0);
            if (v == MAP_FAILED) {
                ::close(fd);
                throw std::runtime_error("cannot map " + path);
            }
            madvise(v, n, MADV_SEQUENTIAL | MADV_WILLNEED);
            p = static_cast<const char*>(v);
        }
        ::close(fd);
    }
    ~Mapped() {
        if (p) munmap(const_cast<char*>(p), n);
    }
};

template <class T>
void exclusive_scan_into(std::vector<uint64_t>& off, const std::vector<T>& cnt) {
    off.assign(cnt.size() + 1, 0);
    for (size_t i = 0; i < cnt.size(); ++i) off[i + 1] = off[i] + (uint64_t)cnt[i];
}

void flat_resize(EigenFlat& F, const std::vector<uint32_t>& k) {
    exclusive_scan_into(F.off, k);
    std::vector<uint64_t> km(k.size());
    for (size_t r = 0; r < k.size(); ++r) km[r] = (uint64_t)k[r] * (uint64_t)std::max(F.m[r], 0);
    exclusive_scan_into(F.eval_off, F.m);
    exclusive_scan_into(F.evec_off, km);
    F.movies.resize(F.off.back());
    F.sigs.resize(F.off.back());
    F.evals.resize(F.eval_off.back());
    if (F.binary) F.evecs_f32.resize(F.evec_off.back());
    else F.evecs.resize(F.evec_off.back());
}

void load_flat_binary(const Mapped& f, const std::string& path, int T, EigenFlat& F) {
    size_t pos = sizeof(kEigenMagic);
    auto need = [&](size_t bytes) {
        if (pos + bytes > f.n) throw std::runtime_error("truncated binary out_eigen_ " + path);
    };
    need(sizeof(uint64_t));
    uint64_t n = 0;
    std::memcpy(&n, f.p + pos, sizeof(n));
    pos += sizeof(n);
    // hop over the record headers: uid k m, then k movies, k sigs, m evals, k*m evecs (4 B each)
    std::vector<size_t> at(n);
    std::vector<uint32_t> k(n);
    F.user.resize(n);
    F.m.resize(n);
    for (uint64_t r = 0; r < n; ++r) {
        uint32_t hdr[3];
        need(sizeof(hdr));
        std::memcpy(hdr, f.p + pos, sizeof(hdr));
        F.user[r] = hdr[0];
        k[r] = hdr[1];
        F.m[r] = (int32_t)hdr[2];
        at[r] = pos + sizeof(hdr);
        const size_t body = 4 * ((size_t)2 * hdr[1] + hdr[2] + (size_t)hdr[1] * hdr[2]);
        need(sizeof(hdr) + body);
        pos += sizeof(hdr) + body;
    }
    F.binary = true;
    flat_resize(F, k);
    if (n == 0) return;
    // record ranges of about equal bytes per thread; the fp32 blocks are copied as they are
    // (the predictor's fp32 entry widens them on the device, exactly)
    std::vector<size_t> cut(T + 1, n);
    cut[0] = 0;
    {
        const size_t total = pos - at.front() + 12, per = total / T + 1;
        size_t t = 1;
        for (size_t r = 0; r < n && t < (size_t)T; ++r)
            if (at[r] - at[0] >= per * t) cut[t++] = r;
        for (; t < (size_t)T; ++t) cut[t] = n;
    }
    parallel_for(T, [&](int t) {
        for (size_t r = cut[t]; r < cut[t + 1]; ++r) {
            const char* q = f.p + at[r];
            const size_t kk = k[r], mm = (size_t)F.m[r];
            std::memcpy(F.movies.data() + F.off[r], q, 4 * kk);
            q += 4 * kk;
            auto widen = [&](double* dst, size_t cnt) {
                for (size_t i = 0; i < cnt; ++i) {
                    float v;
                    std::memcpy(&v, q + 4 * i, 4);
                    dst[i] = v;
                }
                q += 4 * cnt;
            };
            widen(F.sigs.data() + F.off[r], kk);
            widen(F.evals.data() + F.eval_off[r], mm);
            std::memcpy(F.evecs_f32.data() + F.evec_off[r], q, 4 * kk * mm);
        }
    });
}

void load_flat_text(const Mapped& f, const std::string& path, int T, EigenFlat& F) {
    // non-empty line spans, found in parallel over byte ranges
    std::vector<std::vector<const char*>> lb(T), le(T);
    parallel_for(T, [&](int t) {
        const char* beg = f.p + f.n * t / T;
        const char* end = f.p + f.n * (t + 1) / T;
        // a range owns the lines that START in it
        if (t > 0 && beg[-1] != '\n') {
            const char* nl = static_cast<const char*>(std::memchr(beg, '\n', (size_t)(f.p + f.n - beg)));
            beg = nl ? nl + 1 : f.p + f.n;
        }
        const char* fe = f.p + f.n;
        const char* p = beg;
        while (p < end) {
            const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(fe - p)));
            if (!nl) nl = fe;
            if (nl > p) {
                lb[t].push_back(p);
                le[t].push_back(nl);
            }
            p = nl + 1;
        }
    });
    std::vector<const char*> B, E;
    for (int t = 0; t < T; ++t) {
        B.insert(B.end(), lb[t].begin(), lb[t].end());
        E.insert(E.end(), le[t].begin(), le[t].end());
    }
    const size_t n = B.size() / 3;   // a trailing partial record is dropped (state machine)
    std::vector<uint32_t> k(n);
    F.user.resize(n);
    F.m.resize(n);
    std::vector<char> bad(T, 0);
    parallel_for(T, [&](int t) {   // "uid k m" of every record
        for (size_t r = n * t / T; r < n * (t + 1) / T; ++r) {
            Tok tk{B[3 * r], E[3 * r]};
            uint32_t mm = 0;
            if (!tk.u32(F.user[r]) || !tk.u32(k[r]) || !tk.u32(mm)) bad[t] = 1;
            F.m[r] = (int32_t)mm;
        }
    });
    for (char b : bad)
        if (b) throw std::runtime_error("malformed out_eigen_ record in " + path);
    flat_resize(F, k);
    parallel_for(T, [&](int t) {
        for (size_t r = n * t / T; r < n * (t + 1) / T; ++r) {
            const size_t kk = k[r], mm = (size_t)F.m[r];
            bool ok = true;
            Tok a{B[3 * r], E[3 * r]};
            uint32_t skip;
            a.u32(skip), a.u32(skip), a.u32(skip);
            for (size_t i = 0; i < kk; ++i)   // movie sig pairs (:426-442)
                ok &= a.u32(F.movies[F.off[r] + i]) && a.f64(F.sigs[F.off[r] + i]);
            Tok b{B[3 * r + 1], E[3 * r + 1]};   // m eigenvalues (:444-452)
            for (size_t i = 0; i < mm; ++i) ok &= b.f64(F.evals[F.eval_off[r] + i]);
            Tok c{B[3 * r + 2], E[3 * r + 2]};   // k x m eigenvectors (:454-476)
            double* dst = F.evecs.data() + F.evec_off[r];
            for (size_t i = 0; i < kk * mm; ++i) ok &= c.f64(dst[i]);
            if (!ok) bad[t] = 1;   // the reference asserts (:434, 447, 462)
        }
    });
    for (char b : bad)
        if (b) throw std::runtime_error("malformed out_eigen_ record in " + path);
}

}  // namespace

EigenFlat load_eigen_flat(const std::string& path, int n_threads) {
    EigenFlat F;
    const int T = resolve_threads(n_threads);
    bool binary = false;
    {
        std::ifstream h(path, std::ifstream::binary);
        char magic[sizeof(kEigenMagic)] = {};
        binary = h.read(magic, sizeof(magic)) && std::memcmp(magic, kEigenMagic, sizeof(kEigenMagic)) == 0;
    }
    Mapped f(path, !binary);   // the binary form is faulted in by its copying threads
    if (binary)
        load_flat_binary(f, path, T, F);
    else
        load_flat_text(f, path, T, F);
    if (F.off.empty()) {   // no records
        F.off.assign(1, 0);
        F.eval_off.assign(1, 0);
        F.evec_off.assign(1, 0);
    }
    return F;
}

void write_eigen_file(const std::string& path, bool append, int n_threads, bool binary, uint32_t n_users,
                      const uint32_t* uid, const uint64_t* off, const int32_t* m, const uint32_t* movies,
                      const float* sigs, const float* evals, const uint64_t* eoff, const float* evecs) {
    std::ofstream f(path, std::ofstream::binary | (append ? std::ofstream::app : std::ofstream::trunc));
    if (!f) throw std::runtime_error("cannot open " + path);
    if (binary) {
        // "CFEIGEN1", n, then per record uid k m movies[k] sigs[k] evals[m] evecs[k*m]: every
        // record's offset is known from (k, m) up front, so threads pwrite() user ranges in place
        std::vector<uint64_t> at((size_t)n_users + 1, sizeof(kEigenMagic) + sizeof(uint64_t));
        for (uint32_t u = 0; u < n_users; ++u) {
            const uint64_t k = off[u + 1] - off[u], mm = (uint64_t)std::max(m[u], 0);
            at[u + 1] = at[u] + 4 * (3 + 2 * k + mm + k * mm);
        }
        // appended records follow the file's current end (its header, with the total count,
        // was written by start_eigen_file); otherwise the file is this call's records alone
        const uint64_t n = n_users;
        if (!append) {
            f.write(kEigenMagic, sizeof(kEigenMagic));
            f.write(reinterpret_cast<const char*>(&n), sizeof(n));
        }
        f.close();
        const int wfd = ::open(path.c_str(), O_WRONLY);
        if (wfd < 0) throw std::runtime_error("cannot open " + path);
        const uint64_t base = append ? (uint64_t)::lseek(wfd, 0, SEEK_END) - at[0] : 0;
        // the file gets its final size first, so the pieces land inside it instead of extending
        // it out of order; pieces of ~8 MB are claimed in file order by whichever thread is free
        // (a static split by user count left threads idle on unequal byte ranges)
        if (::ftruncate(wfd, (off_t)(base + at[n_users])) != 0) {
            ::close(wfd);
            throw std::runtime_error("cannot size " + path);
        }
        std::vector<uint32_t> piece{0};
        for (uint32_t u = 0; u < n_users;) {
            uint32_t c1 = u + 1;
            while (c1 < n_users && at[c1 + 1] - at[u] < (8u << 20)) ++c1;
            piece.push_back(c1);
            u = c1;
        }
        const uint32_t n_pieces = (uint32_t)piece.size() - 1;
        const int T = (int)std::min<uint32_t>((uint32_t)resolve_threads(n_threads), std::max<uint32_t>(n_pieces, 1));
        std::atomic<bool> failed{false};
        std::atomic<uint32_t> next{0};
        parallel_for(T, [&](int) {
            std::vector<char> buf;
            for (;;) {
                const uint32_t pc = next.fetch_add(1);
                if (pc >= n_pieces) break;
                const uint32_t c0 = piece[pc], c1 = piece[pc + 1];
                buf.resize(at[c1] - at[c0]);
                char* p = buf.data();
                for (uint32_t u = c0; u < c1; ++u) {
                    const uint32_t k = (uint32_t)(off[u + 1] - off[u]), mm = (uint32_t)std::max(m[u], 0);
                    const uint32_t hdr[3] = {uid[u], k, mm};
                    std::memcpy(p, hdr, sizeof(hdr));
                    p += sizeof(hdr);
                    std::memcpy(p, movies + off[u], 4ull * k);
                    p += 4ull * k;
                    std::memcpy(p, sigs + off[u], 4ull * k);
                    p += 4ull * k;
                    for (uint32_t j = 0; j < mm; ++j) {   // entries past k (k == 1 padding) are 0
                        const float v = j < k ? evals[off[u] + j] : 0.0f;
                        std::memcpy(p, &v, 4);
                        p += 4;
                    }
                    std::memcpy(p, evecs + eoff[u], 4ull * k * mm);
                    p += 4ull * k * mm;
                }
                size_t done = 0;
                while (done < buf.size()) {
                    const ssize_t w = ::pwrite(wfd, buf.data() + done, buf.size() - done, (off_t)(base + at[c0] + done));
                    if (w <= 0) {
                        failed = true;
                        break;
                    }
                    done += (size_t)w;
                }
                if (failed) break;
            }
        });
        ::close(wfd);
        if (failed) throw std::runtime_error("write failed: " + path);
        return;
    }
    // text: chunks of users formatted in parallel; chunk c lands at the sum of the sizes of
    // chunks 0..c-1, published along a chain as soon as each chunk is formatted, and every
    // thread pwrite()s its own chunk there -- formatting and writing overlap, no serial writer
    f.close();   // created (or truncated) above; appended records start at its current end
    const int wfd = ::open(path.c_str(), O_WRONLY);
    if (wfd < 0) throw std::runtime_error("cannot open " + path);
    const uint64_t base = append ? (uint64_t)::lseek(wfd, 0, SEEK_END) : 0;
    const int T = (int)std::min<uint32_t>((uint32_t)resolve_threads(n_threads), std::max<uint32_t>(n_users, 1));
    const uint32_t chunk = 256;    // users per formatting task (~4-8 MB of text at k ~ 100)
    const uint32_t n_chunks = (n_users + chunk - 1) / chunk;
    std::vector<uint64_t> start(n_chunks + 1, 0);
    std::vector<std::atomic<int>> ready(n_chunks + 1);
    for (auto& r : ready) r.store(0);
    ready[0].store(1);
    std::atomic<bool> failed{false};
    std::atomic<uint32_t> next{0};
    parallel_for(T, [&](int) {
        std::string buf;
        for (;;) {
            const uint32_t c = next.fetch_add(1);
            if (c >= n_chunks) break;
            buf.clear();
            const uint32_t u0 = c * chunk, u1 = std::min(n_users, u0 + chunk);
            uint64_t vals = 0;
            for (uint32_t u = u0; u < u1; ++u) {
                const uint64_t k = off[u + 1] - off[u];
                vals += 2 * k + (uint64_t)m[u] * (k + 1);
            }
            buf.reserve(12 * vals + 64);   // %g of 6 digits + sign + separator
            for (uint32_t u = u0; u < u1; ++u) {
                const uint32_t k = (uint32_t)(off[u + 1] - off[u]);
                append_eigen_record(buf, uid[u], k, (uint32_t)m[u], movies + off[u], sigs + off[u], evals + off[u],
                                    evecs + eoff[u]);
            }
            // chunks are claimed in order, so the chain below waits only on formatting in flight
            while (!ready[c].load(std::memory_order_acquire)) std::this_thread::yield();
            start[c + 1] = start[c] + buf.size();
            ready[c + 1].store(1, std::memory_order_release);
            size_t done = 0;
            while (done < buf.size()) {
                const ssize_t w = ::pwrite(wfd, buf.data() + done, buf.size() - done, (off_t)(base + start[c] + done));
                if (w <= 0) {
                    failed = true;
                    break;
                }
                done += (size_t)w;
            }
        }
    });
    ::close(wfd);
    if (failed) throw std::runtime_error("write failed: " + path);
}

void start_eigen_file(const std::string& path, bool binary, uint64_t n_total) {
    std::ofstream f(path, std::ofstream::binary | std::ofstream::trunc);
    if (!f) throw std::runtime_error("cannot open " + path);
    if (binary) {
        f.write(kEigenMagic, sizeof(kEigenMagic));
        f.write(reinterpret_cast<const char*>(&n_total), sizeof(n_total));
    }
    if (!f) throw std::runtime_error("write failed: " + path);
}

}  // namespace cfio

// C entry points used by the Python side (tests compare the formatting with printf, and the
// parallel / binary out_eigen_ writers and readers with the serial text form).
extern "C" int cfh_start_eigen(const char* path, int binary, uint64_t n_total) {
    try {
        cfio::start_eigen_file(path, binary != 0, n_total);
    } catch (const std::exception&) {
        return -1;
    }
    return 0;
}

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
        const auto F = cfio::load_eigen_flat(path, n_threads);
        if (!flat) return (int64_t)F.size();
        int64_t pos = 0;
        auto put = [&](double v) {
            if (flat && pos < cap) flat[pos] = v;
            ++pos;
        };
        for (size_t r = 0; r < F.size(); ++r) {
            const uint64_t k = F.off[r + 1] - F.off[r];
            put(F.user[r]);
            put((double)k);
            put((double)F.m[r]);
            for (uint64_t i = F.off[r]; i < F.off[r + 1]; ++i) put(F.movies[i]);
            for (uint64_t i = F.off[r]; i < F.off[r + 1]; ++i) put(F.sigs[i]);
            for (uint64_t i = F.eval_off[r]; i < F.eval_off[r + 1]; ++i) put(F.evals[i]);
            for (uint64_t i = F.evec_off[r]; i < F.evec_off[r + 1]; ++i)
                put(F.binary ? (double)F.evecs_f32[i] : F.evecs[i]);
        }
        if (flat && pos > cap) return -2;
        return (int64_t)F.size();
    } catch (const std::exception&) {
        return -1;
    }
}

// Formatting / parsing probes for tests/test_formats.py: format_g6 (the writers' %g) and
// parse_f64 (the readers' strtod) over arrays.
extern "C" int64_t cfh_format_many(const double* v, int64_t n, char* out, int64_t cap) {
    int64_t pos = 0;
    char buf[64];
    for (int64_t i = 0; i < n; ++i) {
        char* e = cfio::format_g6(buf, v[i]);
        const int64_t len = e - buf;
        if (pos + len + 1 > cap) return -1;
        std::memcpy(out + pos, buf, (size_t)len);
        pos += len;
        out[pos++] = '\n';
    }
    return pos;
}

extern "C" int64_t cfh_parse_many(const char* text, int64_t len, double* out, int64_t cap) {
    const char* p = text;
    const char* e = text + len;
    int64_t n = 0;
    while (p < e && n < cap) {
        while (p < e && (*p == ' ' || *p == '\n')) ++p;
        if (p >= e) break;
        if (!cfio::parse_f64(p, e, out[n])) return -1;
        ++n;
    }
    return n;
}

// C entry points used by the Python side (tests compare the formatting with printf).
extern "C" int cfh_format_g(double v, char* buf, int cap) {
    std::string s;
    cfio::append_g(s, v);
    if ((int)s.size() + 1 > cap) return -1;
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return (int)s.size();
}
