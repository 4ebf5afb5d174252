// cf_io.hpp -- the reference's CWD text-file contract in C++.
//
// Files are whitespace-separated ASCII; numbers use the iostream defaults of the
// reference (%g, 6 significant digits).  GraphLab's graph.save writes
// "<prefix>_<i>_of_<N>" shards (evidence: extract_user.py:7-10); the shard a vertex
// lands in is unpinned upstream, here it is (id % N) + 1 and lines are in ascending
// id order.
#pragma once

#include <cstdint>
#include <string>
#include <memory>
#include <unordered_map>
#include <utility>
#include <vector>

namespace cfio {

constexpr uint32_t kUimax = 2147483647u;  // std::numeric_limits<int>::max() as unsigned (knn.cpp:19)

// Sorted regular files in `dir` whose name ends with / starts with the given string
// (list_files_with_suffix / _prefix, precompute_local_threads.cpp:42-87).
std::vector<std::string> files_with_suffix(const std::string& dir, const std::string& suffix);
std::vector<std::string> files_with_prefix(const std::string& dir, const std::string& prefix);
std::string read_file(const std::string& path);

// %g with precision 6, exactly as `std::ostream << double` with default flags.
void append_g(std::string& out, double v);
char* format_g6(char* p, double v);                        // the same into p, returns the end
bool parse_f64(const char*& p, const char* e, double& out);   // strtod-exact decimal parse
void append_u(std::string& out, uint64_t v);

// A movielens rating triplet (user id already remapped to uimax - uid where asked).
struct Rating {
    uint32_t user;
    uint32_t movie;
    double value;
    bool validate;
};

// movielens/*: role VALIDATE if the file name ends with ".validate", else TRAIN
// (knn.cpp:88-92); source id remapped to uimax - id (knn.cpp:103).
std::vector<Rating> load_movielens(const std::string& dir, bool remap_users);

// Per-vertex lines "id a b a b ..." (out_rat_, out_test_rat_): id -> [(user, rating)].
using VertexRatings = std::unordered_map<uint32_t, std::vector<std::pair<uint32_t, double>>>;
VertexRatings load_vertex_ratings(const std::string& dir, const std::string& prefix,
                                  bool require_nonempty);

// Edge lines "a b w" (out_fin_).  Keeps the last occurrence of a duplicate pair.
struct Edge {
    uint32_t a, b;
    double w;
};
std::vector<Edge> load_edges(const std::string& dir, const std::string& prefix);

// Adjacency lines "a b c d ..." (out_edg_).
std::vector<std::pair<uint32_t, uint32_t>> load_adjacency(const std::string& dir,
                                                          const std::string& prefix);

// Sharded writer: line for vertex `id` goes to <prefix>_<(id % n)+1>_of_<n>.
class ShardWriter {
   public:
    ShardWriter(const std::string& dir, const std::string& prefix, int nshards);
    std::string& shard(uint32_t id) { return buf_[id % buf_.size()]; }
    void flush();

   private:
    std::string dir_, prefix_;
    std::vector<std::string> buf_;
};

// Compact id space: sorted unique ids -> 0..n-1.
struct IdMap {
    std::vector<uint32_t> ids;                 // compact -> id
    std::unordered_map<uint32_t, uint32_t> at; // id -> compact
    void build(std::vector<uint32_t> all);
    uint32_t size() const { return (uint32_t)ids.size(); }
};

// out_eigen_ record writer (README.md:14-19; precompute_local_threads.cpp:196-210).
void append_eigen_record(std::string& out, uint32_t user, uint32_t k, uint32_t m,
                         const uint32_t* movies, const float* sigs, const float* evals,
                         const float* evecs);
// load_precomputed_data (local_calc_precomp.cpp:406-482; its 3-line state machine for text, or
// the "CFEIGEN1" binary form of write_eigen_file) straight into flat arrays (no per-record
// vectors): the file is mapped,
// record boundaries found in parallel, and every record parsed (text) or widened (binary) into
// its place on n_threads threads.  Record r of the n in file order: user[r], k = off[r+1] -
// off[r] movies / sigs at off[r], m[r] eigenvalues at eval_off[r], its k x m row-major block at
// evec_off[r].
// Allocator whose resize() leaves elements uninitialised: the loader's threads write (first
// touch) every element of the big arrays themselves instead of one thread zeroing them first.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        if constexpr (sizeof...(A) == 0) ::new ((void*)p) U;
        else ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
template <class T>
using RawVec = std::vector<T, NoInitAlloc<T>>;

struct EigenFlat {
    std::vector<uint32_t> user;
    std::vector<uint64_t> off;        // n + 1, prefix of k
    std::vector<int32_t> m;
    RawVec<uint32_t> movies;
    RawVec<double> sigs;
    std::vector<uint64_t> eval_off;   // n + 1, prefix of m
    RawVec<double> evals;
    std::vector<uint64_t> evec_off;   // n + 1, prefix of k * m
    RawVec<double> evecs;             // text form (decimal %g values parse to double, :454-476)
    RawVec<float> evecs_f32;          // binary form: the file's fp32 blocks, copied as they are
    bool binary = false;              // evecs_f32 holds the blocks (else evecs)
    size_t size() const { return user.size(); }
};
EigenFlat load_eigen_flat(const std::string& path, int n_threads = 0);
// out_eigen_ writer (precompute_local_threads.cpp:196-211): text records formatted on
// n_threads threads (contiguous user ranges, written in user order), or the binary form
// (the reference's own TODO, README.md:29).  eoff[u] locates user u's k x m
// block in evecs (slot offsets or packed offsets alike).  append: the records follow the
// file's end (binary: no header of their own, see start_eigen_file).
void write_eigen_file(const std::string& path, bool append, int n_threads, bool binary, uint32_t n_users,
                      const uint32_t* uid, const uint64_t* off, const int32_t* m, const uint32_t* movies,
                      const float* sigs, const float* evals, const uint64_t* eoff, const float* evecs);
// A file written in pieces (bin/precompute_local's chunks, in user order): start_eigen_file
// truncates it and, for the binary form, writes the header with the total record count; every
// piece is then write_eigen_file(append = true).  The bytes equal one write_eigen_file over all
// records.
void start_eigen_file(const std::string& path, bool binary, uint64_t n_total);

}  // namespace cfio
