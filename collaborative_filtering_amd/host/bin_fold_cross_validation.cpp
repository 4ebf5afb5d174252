// fold_cross_validation -- drop-in for fold_cross_validation.py.
//   :8-22   read "user \t item \t rating ..." lines into data[user] (users in first-appearance
//           order, each user's (item, rating) list in line order; ints as parsed by int())
//   :25-26  mkdir cross_validation (an existing directory is an error, as os.mkdir)
//   :32-46  keys shuffled by random.shuffle; users appended to fold `ind` until
//           n_usr_done > num_usr / num_div (true division), then the next fold
//   :48-57  u<i>.test = fold i, u<i>.train = every other fold in fold order
// The shuffle is CPython's (cf_pyrand.hpp) under random.seed(--seed), so a seeded run of the
// script and this binary write identical files.  The ratings are grouped by the users'
// shuffled ranks on the GPU (cf_fold_order: one stable radix sort).
// Usage: fold_cross_validation <file> <num_div> [--seed S] (default seed: time)
#include <sys/stat.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <unordered_map>

#include "cf_cli.hpp"
#include "cf_pyrand.hpp"

static bool parse_int(const char*& p, const char* e, int64_t& v) {   // int(): surrounding whitespace
    while (p < e && (*p == ' ' || *p == '\r' || *p == '\n' || *p == '\v' || *p == '\f')) ++p;
    bool neg = false;
    if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
    if (p >= e || *p < '0' || *p > '9') return false;
    v = 0;
    while (p < e && *p >= '0' && *p <= '9') v = v * 10 + (*p++ - '0');
    if (neg) v = -v;
    while (p < e && (*p == ' ' || *p == '\r' || *p == '\n' || *p == '\v' || *p == '\f')) ++p;
    return true;
}

int main(int argc, char** argv) {
    if (argc < 3 || argv[1][0] == '-') cfcli::die("usage: fold_cross_validation <file> <num_div> [--seed S]");
    const std::string path = argv[1];
    const int64_t num_div = std::atoll(argv[2]);
    if (num_div <= 0) cfcli::die("num_div must be positive");
    const uint64_t seed = std::stoull(cfcli::opt(argc, argv, "seed", std::to_string((uint64_t)std::time(nullptr))));

    const std::string text = cfio::read_file(path);
    std::unordered_map<int64_t, uint32_t> uid;
    std::vector<int64_t> keys;                    // users, first-appearance order
    std::vector<uint32_t> user;                   // per line: compact user
    std::vector<int64_t> item, rating;
    const char* p = text.data();
    const char* end = p + text.size();
    while (p < end) {
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', end - p));
        const char* le = nl ? nl : end;
        // val = line.split('\t'); int(val[0]), int(val[1]), int(val[2])
        const char* f[3];
        const char* fe[3];
        const char* q = p;
        int nf = 0;
        for (; nf < 3; ++nf) {
            f[nf] = q;
            const char* t = static_cast<const char*>(std::memchr(q, '\t', le - q));
            fe[nf] = t ? t : le;
            if (!t) {
                ++nf;
                break;
            }
            q = t + 1;
        }
        if (nf < 3) cfcli::die("line without three tab-separated fields");
        int64_t v[3];
        for (int i = 0; i < 3; ++i) {
            const char* a = f[i];
            if (!parse_int(a, fe[i], v[i]) || a < fe[i])
                cfcli::die("non-integer field");
        }
        auto it = uid.find(v[0]);
        if (it == uid.end()) {
            it = uid.emplace(v[0], (uint32_t)keys.size()).first;
            keys.push_back(v[0]);
        }
        user.push_back(it->second);
        item.push_back(v[1]);
        rating.push_back(v[2]);
        p = nl ? nl + 1 : end;
    }
    const uint32_t num_usr = (uint32_t)keys.size();

    std::vector<uint32_t> perm(num_usr);   // keys = list(data.keys()); random.shuffle(keys)
    for (uint32_t i = 0; i < num_usr; ++i) perm[i] = i;
    pyrand::MT(seed).shuffle(perm);
    std::vector<uint32_t> rank(num_usr), fold_of_rank(num_usr);
    int64_t ind = 0, done = 0;
    const double per = (double)num_usr / (double)num_div;
    for (uint32_t r = 0; r < num_usr; ++r) {
        rank[perm[r]] = r;
        fold_of_rank[r] = (uint32_t)ind;
        if (++done > per) {
            done = 0;
            ++ind;
        }
    }
    const int64_t n_folds = ind + 1;

    std::vector<uint32_t> order(user.size());
    cf_ctx* ctx = cfcli::open_device();
    cfcli::check(ctx, cf_fold_order(ctx, user.size(), num_usr, user.data(), rank.data(), order.data()), "cf_fold_order");
    cf_destroy(ctx);

    std::vector<std::string> test(n_folds);
    for (uint32_t i : order) {
        std::string& out = test[fold_of_rank[rank[user[i]]]];
        out += std::to_string(keys[user[i]]);
        out += '\t';
        out += std::to_string(item[i]);
        out += '\t';
        out += std::to_string(rating[i]);
        out += '\n';
    }
    if (mkdir("cross_validation", 0777) != 0)
        cfcli::die(std::string("mkdir cross_validation: ") + std::strerror(errno));
    for (int64_t i = 0; i < n_folds; ++i) {
        const std::string base = "cross_validation/u" + std::to_string(i);
        FILE* ft = std::fopen((base + ".test").c_str(), "wb");
        FILE* fr = std::fopen((base + ".train").c_str(), "wb");
        if (!ft || !fr) cfcli::die("cannot write " + base);
        std::fwrite(test[i].data(), 1, test[i].size(), ft);
        for (int64_t j = 0; j < n_folds; ++j)
            if (j != i) std::fwrite(test[j].data(), 1, test[j].size(), fr);
        std::fclose(ft);
        std::fclose(fr);
    }
    std::printf("%u users, %zu ratings -> %lld folds in cross_validation/\n", num_usr, user.size(), (long long)n_folds);
    return 0;
}
