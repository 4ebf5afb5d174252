// cf_prep.hip -- GPU data prep: the knn regroup and the
// user-disjoint k-fold split, as sorts and bitmaps in HBM instead of hash-map merges.
//
// knn regroup (knn.cpp:83-357).  The reference loads user -> movie edges with a role
// (TRAIN / VALIDATE by file suffix, :88-92) and runs three GraphLab programs:
//   vertex_program  (:160-205)  movie gathers its in-edges into `ratings` (train) and
//                               `ratings_test` (validate) maps -> out_rat_ / out_test_rat_
//   vertex2/3       (:212-298)  user collects its movies, movie unions its raters' sets
//                               (both roles, :224-227, 271-274) -> out_edg_ (sorted, :342-351)
// Here, over the ratings in read order (compact ids):
//   1. key = (role * n_movies + movie) << 32 | user, stable LSD radix sort of (key, index):
//      equal keys keep read order, so the LAST rating of a (role, movie, user) -- the map
//      assignment semantics -- is the last of its run; a flag + exclusive scan keeps it and
//      the runs land grouped by role, then movie, users ascending: the two CSR lists;
//   2. key = user << 32 | movie, sorted and made unique: every user's movie set (CSR);
//   3. co-rated bitmap n_movies x ceil(n_movies / 32) words: per user, every pair (a, b) of
//      its set ORs bit b into row a -- the sorted set puts equal words in adjacent lanes,
//      so a segmented OR over the wave leaves one atomicOr per (a, 32-column word);
//   4. row popcounts (self bit cleared), exclusive scan, and a block scan per row that
//      writes the set bits in ascending order: the sorted unique co-rated lists.
// Bytes: ~40 B per rating through the two sorts plus n_movies^2 / 8 of bitmap; the pair
// ORs are sum_u deg_u^2 atomics spread over the bitmap (L2-resident up to ~30k movies).
//
// k-fold split (fold_cross_validation.py:31-57): the host shuffles the users (Python's
// random.shuffle, reproduced bit for bit in the binary) and hands each user its rank;
// the ratings are ordered by (rank, read order) with one stable radix sort of rank keys.
// The folds are contiguous rank ranges of that order (the host computes the boundaries
// with the script's `n_usr_done > num_usr / num_div` rule).

#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>

#include "cf_internal.h"

namespace {

// Sorts run rocprim's stable merge-sort path at every size (radix_sort_config with an unbounded
// merge-sort limit).  Inside a PyTorch process this library is served by torch's bundled HIP
// runtime, under which rocprim's onesweep radix path fails to launch (hipErrorInvalidValue, in
// both its gfx950-tuned and generic configurations), while the merge path runs; standalone on
// the ROCm 7.2 runtime all of them run (tools/probe_sort.hip, 10.7M u64 keys + u32 values,
// 47 bits: onesweep 0.94 ms, merge sort 0.86 ms).
using SortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config,
                                           (size_t)1 << 40>;

template <class K, class V>
hipError_t sort_pairs(void* tmp, size_t& bytes, const K* ki, K* ko, const V* vi, V* vo, uint64_t n, int bits,
                      hipStream_t st) {
    return rocprim::radix_sort_pairs<SortCfg>(tmp, bytes, ki, ko, vi, vo, (unsigned int)n, 0u, (unsigned int)bits, st);
}
template <class K>
hipError_t sort_keys(void* tmp, size_t& bytes, const K* ki, K* ko, uint64_t n, int bits, hipStream_t st) {
    return rocprim::radix_sort_keys<SortCfg>(tmp, bytes, ki, ko, (unsigned int)n, 0u, (unsigned int)bits, st);
}

inline int bits_for(uint64_t n) {   // bits to represent 0 .. n-1 (>= 1)
    int b = 1;
    while (b < 64 && (1ull << b) < n) ++b;
    return b;
}

__global__ void regroup_keys_kernel(uint64_t n, const uint32_t* user, const uint32_t* movie, const uint8_t* role,
                                    uint32_t n_movies, uint64_t* key, uint32_t* idx) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t seg = (role && role[i]) ? (uint64_t)n_movies + movie[i] : movie[i];
        key[i] = seg << 32 | user[i];
        idx[i] = (uint32_t)i;
    }
}

// keep[i] = 1 for the last element of a run of equal keys (last read wins) or, with
// first != 0, for the first element of a run (set semantics)
__global__ void run_flag_kernel(uint64_t n, const uint64_t* key, int first, uint32_t* keep) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        keep[i] = first ? (i == 0 || key[i] != key[i - 1]) : (i + 1 == n || key[i + 1] != key[i]);
}

// kept element j = pos[i] of segment seg = key >> 32: counted per segment, its user and
// rating stored at j (positions are already grouped by segment: the keys are sorted)
__global__ void regroup_scatter_kernel(uint64_t n, const uint64_t* key, const uint32_t* idx, const uint32_t* keep,
                                       const uint32_t* pos, const float* rating, uint32_t* seg_cnt, uint32_t* out_user,
                                       float* out_rating) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (!keep[i]) continue;
        const uint64_t k = key[i];
        const uint32_t j = pos[i];
        atomicAdd(&seg_cnt[k >> 32], 1u);
        out_user[j] = (uint32_t)k;
        out_rating[j] = rating[idx[i]];
    }
}

// seg_off (2 n_movies + 1) -> train_off[m] = seg_off[m], test_off[m] = seg_off[n_movies + m]
// - seg_off[n_movies]; the kept (user, rating) pairs split at seg_off[n_movies]
__global__ void regroup_split_kernel(uint32_t n_movies, const uint64_t* seg_off, uint64_t* train_off,
                                     uint64_t* test_off, const uint32_t* kuser, const float* krat, uint32_t* tr_user,
                                     float* tr_rat, uint32_t* te_user, float* te_rat) {
    const uint64_t ntr = seg_off[n_movies], ntot = seg_off[2 * (uint64_t)n_movies];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t m = t0; m <= n_movies; m += stride) {
        train_off[m] = seg_off[m];
        test_off[m] = seg_off[n_movies + m] - ntr;
    }
    for (uint64_t j = t0; j < ntot; j += stride) {
        if (j < ntr) {
            tr_user[j] = kuser[j];
            tr_rat[j] = krat[j];
        } else {
            te_user[j - ntr] = kuser[j];
            te_rat[j - ntr] = krat[j];
        }
    }
}

__global__ void user_keys_kernel(uint64_t n, const uint32_t* user, const uint32_t* movie, uint64_t* key) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        key[i] = (uint64_t)user[i] << 32 | movie[i];
}

__global__ void user_sets_kernel(uint64_t n, const uint64_t* key, const uint32_t* keep, const uint32_t* pos,
                                 uint32_t* ucnt, uint32_t* list) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (!keep[i]) continue;
        atomicAdd(&ucnt[key[i] >> 32], 1u);
        list[pos[i]] = (uint32_t)key[i];
    }
}

// One workgroup per user: for each row a of its (sorted) movie set, the wave ORs the bits
// of every b of the set into row a.  Lanes holding the same 32-column word are adjacent;
// a suffix OR over equal-word lanes leaves the segment's bits in its first lane, which
// issues the one atomic of that word.
constexpr int kPrepThreads = 256;
__global__ void __launch_bounds__(kPrepThreads) corated_bits_kernel(uint32_t n_users, const uint64_t* uoff,
                                                                   const uint32_t* list, uint32_t words,
                                                                   uint32_t* bm) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t u = blockIdx.x; u < n_users; u += gridDim.x) {
        const uint64_t s = uoff[u];
        const uint32_t d = (uint32_t)(uoff[u + 1] - s);
        if (d < 2) continue;
        for (uint32_t ia = wave; ia < d; ia += kPrepThreads / 64) {
            const uint32_t a = list[s + ia];
            uint32_t* row = bm + (size_t)a * words;
            for (uint32_t b0 = 0; b0 < d; b0 += 64) {
                const bool ok = b0 + lane < d;
                const uint32_t b = ok ? list[s + b0 + lane] : 0u;
                const uint32_t w = ok ? (b >> 5) : 0xffffffffu;
                uint32_t bits = ok ? (1u << (b & 31)) : 0u;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t vb = __shfl_down(bits, o);
                    const uint32_t vw = __shfl_down(w, o);
                    if (lane + o < 64 && vw == w) bits |= vb;
                }
                const uint32_t wprev = __shfl_up(w, 1);
                if (ok && (lane == 0 || wprev != w)) atomicOr(&row[w], bits);
            }
        }
    }
}

// One wave per movie row: popcount of the row without its self bit.
__global__ void row_count_kernel(uint32_t n_movies, uint32_t words, const uint32_t* bm, uint64_t* cnt) {
    const int lane = threadIdx.x & 63;
    const uint32_t wpb = blockDim.x / 64;
    for (uint32_t a = blockIdx.x * wpb + (threadIdx.x >> 6); a < n_movies; a += gridDim.x * wpb) {
        const uint32_t* row = bm + (size_t)a * words;
        uint32_t c = 0;
        for (uint32_t w = lane; w < words; w += 64) c += __popc(row[w] & (w == (a >> 5) ? ~(1u << (a & 31)) : ~0u));
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        if (lane == 0) cnt[a] = c;
    }
}

// One workgroup per row: the set bits in ascending order at edg_off[a] (writes past cap are
// dropped; the offsets are complete regardless).
__global__ void __launch_bounds__(kPrepThreads) row_write_kernel(uint32_t n_movies, uint32_t words, const uint32_t* bm,
                                                                const uint64_t* off, uint32_t* col, uint64_t cap) {
    using Scan = hipcub::BlockScan<uint32_t, kPrepThreads>;
    __shared__ typename Scan::TempStorage tmp;
    __shared__ uint32_t s_run;
    for (uint32_t a = blockIdx.x; a < n_movies; a += gridDim.x) {
        const uint32_t* row = bm + (size_t)a * words;
        uint64_t base = off[a];
        for (uint32_t w0 = 0; w0 < words; w0 += kPrepThreads) {
            const uint32_t w = w0 + threadIdx.x;
            uint32_t bits = w < words ? row[w] : 0u;
            if (w == (a >> 5)) bits &= ~(1u << (a & 31));   // self removed (knn.cpp:342-351)
            uint32_t pre = 0, tot = 0;
            Scan(tmp).ExclusiveSum((uint32_t)__popc(bits), pre, tot);
            uint64_t o = base + pre;
            while (bits) {
                const int t = __ffs(bits) - 1;
                bits &= bits - 1;
                if (o < cap) col[o] = w * 32 + t;
                ++o;
            }
            if (threadIdx.x == 0) s_run = tot;
            __syncthreads();
            base += s_run;
            __syncthreads();
        }
    }
}

__global__ void fold_keys_kernel(uint64_t n, const uint32_t* user, const uint32_t* rank, uint32_t* key, uint32_t* idx) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        key[i] = rank[user[i]];
        idx[i] = (uint32_t)i;
    }
}

inline dim3 grid_for(uint64_t n) { return dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 65536))); }

// Bump allocator over the context's prep scratch (grown to the request, 256 B aligned).
struct Carve {
    char* base;
    size_t used = 0;
    template <class T>
    T* take(size_t count) {
        T* p = reinterpret_cast<T*>(base + used);
        used += (sizeof(T) * std::max<size_t>(count, 1) + 255) & ~size_t(255);
        return p;
    }
};

int prep_reserve(cf_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->prep_bytes) return CF_OK;
    if (ctx->d_prep) (void)hipFree(ctx->d_prep);
    ctx->d_prep = nullptr;
    ctx->prep_bytes = 0;
    if (hipMalloc(&ctx->d_prep, bytes) != hipSuccess) return cf_set_error(ctx, CF_ENOMEM, "prep scratch");
    ctx->prep_bytes = bytes;
    return CF_OK;
}

int prep_events(cf_ctx* ctx) {
    for (hipEvent_t& e : ctx->prep_ev)
        if (!e) CF_HIP_CHECK(ctx, hipEventCreate(&e));
    return CF_OK;
}

// cub temporary-storage sizes, queried with exactly the arguments of the real calls (rocprim
// sizes its onesweep storage from the bit range and the stream's target)
size_t cub_bytes(uint64_t n, uint64_t nseg, int bits_a, int bits_b, int bits_fold, hipStream_t st) {
    size_t a = 0, b = 0, c = 0, d = 0, e = 0;
    (void)sort_pairs(nullptr, a, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const uint32_t*)nullptr,
                     (uint32_t*)nullptr, n, bits_a, st);
    (void)sort_keys(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr, n, bits_b, st);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, st);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, d, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)nseg, st);
    (void)sort_pairs(nullptr, e, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                     (uint32_t*)nullptr, n, bits_fold, st);
    return std::max({a, b, c, d, e}) + 4096;
}

// widen u32 counts into u64 for the offset scans
__global__ void widen_kernel(uint64_t n, const uint32_t* in, uint64_t* out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

}  // namespace

int cf_knn_regroup_run(cf_ctx* ctx, uint64_t n, uint32_t n_users, uint32_t n_movies, const uint32_t* d_user,
                       const uint32_t* d_movie, const float* d_rating, const uint8_t* d_validate, uint64_t* d_train_off,
                       uint32_t* d_train_user, float* d_train_rating, uint64_t* d_test_off, uint32_t* d_test_user,
                       float* d_test_rating, uint64_t* d_edg_off, uint32_t* d_edg_movie, uint64_t edg_cap,
                       void* stream_) {
    if (!ctx) return CF_EINVAL;
    if (n >= (1ull << 31) || n_movies >= (1u << 30))
        return cf_set_error(ctx, CF_ERANGE, "cf_knn_regroup_run: more than 2^31 ratings or 2^30 movies");
    if ((n && (!d_user || !d_movie || !d_rating)) || !d_train_off || !d_test_off || !d_edg_off ||
        (n && (!d_train_user || !d_train_rating || !d_test_user || !d_test_rating)) || (edg_cap && !d_edg_movie))
        return cf_set_error(ctx, CF_EINVAL, "cf_knn_regroup_run: null argument");
    CF_TRY(set_device(ctx));
    CF_TRY(prep_events(ctx));
    hipStream_t st = (hipStream_t)stream_;
    const uint64_t nseg = 2 * (uint64_t)n_movies + 1;
    const uint32_t words = (n_movies + 31) / 32;
    const int bits_a = 32 + bits_for(nseg), bits_b = 32 + bits_for((uint64_t)n_users + 1);
    const size_t cub = cub_bytes(n, std::max<uint64_t>(nseg, (uint64_t)n_users + 1), bits_a, bits_b, 1, st);
    // the scratch layout, carved twice: a dry run over a null base sizes the reservation
    // from exactly the takes the real carve makes
    struct Layout {
        uint64_t *key_a, *key_b, *seg_w, *seg_off, *uw, *uoff, *rcnt;
        uint32_t *idx_a, *idx_b, *keep, *pos, *kuser, *seg_cnt, *ucnt, *bm;
        void* tmp;
    };
    const auto carve = [&](char* base, Layout& L) {
        Carve cv{base};
        L.key_a = cv.take<uint64_t>(n);
        L.key_b = cv.take<uint64_t>(n);
        L.idx_a = cv.take<uint32_t>(n);
        L.idx_b = cv.take<uint32_t>(n);
        L.keep = cv.take<uint32_t>(n);
        L.pos = cv.take<uint32_t>(n);
        L.kuser = cv.take<uint32_t>(n);
        L.seg_cnt = cv.take<uint32_t>(nseg);
        L.seg_w = cv.take<uint64_t>(nseg);
        L.seg_off = cv.take<uint64_t>(nseg);
        L.ucnt = cv.take<uint32_t>((uint64_t)n_users + 1);
        L.uw = cv.take<uint64_t>((uint64_t)n_users + 1);
        L.uoff = cv.take<uint64_t>((uint64_t)n_users + 1);
        L.bm = cv.take<uint32_t>((uint64_t)n_movies * words);
        L.rcnt = cv.take<uint64_t>((uint64_t)n_movies + 1);
        L.tmp = cv.take<char>(cub);
        return cv.used;
    };
    Layout lay{};
    const size_t need = carve(nullptr, lay);
    CF_TRY(prep_reserve(ctx, need));
    if (carve(static_cast<char*>(ctx->d_prep), lay) > ctx->prep_bytes)
        return cf_set_error(ctx, CF_EINVAL, "cf_knn_regroup_run: scratch layout exceeds the reservation");
    uint64_t *key_a = lay.key_a, *key_b = lay.key_b, *seg_w = lay.seg_w, *seg_off = lay.seg_off, *uw = lay.uw,
             *uoff = lay.uoff, *rcnt = lay.rcnt;
    uint32_t *idx_a = lay.idx_a, *idx_b = lay.idx_b, *keep = lay.keep, *pos = lay.pos, *kuser = lay.kuser,
             *seg_cnt = lay.seg_cnt, *ucnt = lay.ucnt, *bm = lay.bm;
    float* krat = reinterpret_cast<float*>(idx_a);   // idx_a is dead after the first sort
    void* tmp = lay.tmp;
    size_t tb = cub;
    const dim3 G = grid_for(n), B(256);
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->prep_ev[0], st));
    // ---- 1. per-movie train / test lists ----------------------------------------------
    if (n) {
        hipLaunchKernelGGL(regroup_keys_kernel, G, B, 0, st, n, d_user, d_movie, d_validate, n_movies, key_a, idx_a);
        CF_HIP_CHECK(ctx, hipGetLastError());
        CF_HIP_CHECK(ctx, sort_pairs(tmp, tb, key_a, key_b, idx_a, idx_b, n, bits_a, st));
        hipLaunchKernelGGL(run_flag_kernel, G, B, 0, st, n, key_b, 0, keep);
        CF_HIP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tb, keep, pos, (int)n, st));
    }
    CF_HIP_CHECK(ctx, hipMemsetAsync(seg_cnt, 0, sizeof(uint32_t) * nseg, st));
    if (n)
        hipLaunchKernelGGL(regroup_scatter_kernel, G, B, 0, st, n, key_b, idx_b, keep, pos, d_rating, seg_cnt, kuser,
                           krat);
    hipLaunchKernelGGL(widen_kernel, grid_for(nseg), B, 0, st, nseg, seg_cnt, seg_w);
    CF_HIP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tb, seg_w, seg_off, (int)nseg, st));
    hipLaunchKernelGGL(regroup_split_kernel, grid_for(std::max<uint64_t>(n, n_movies + 1)), B, 0, st, n_movies, seg_off,
                       d_train_off, d_test_off, kuser, krat, d_train_user, d_train_rating, d_test_user, d_test_rating);
    // ---- 2. per-user movie sets (both roles) --------------------------------------------
    CF_HIP_CHECK(ctx, hipMemsetAsync(ucnt, 0, sizeof(uint32_t) * ((uint64_t)n_users + 1), st));
    if (n) {
        hipLaunchKernelGGL(user_keys_kernel, G, B, 0, st, n, d_user, d_movie, key_a);
        CF_HIP_CHECK(ctx, sort_keys(tmp, tb, key_a, key_b, n, bits_b, st));
        hipLaunchKernelGGL(run_flag_kernel, G, B, 0, st, n, key_b, 1, keep);
        CF_HIP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tb, keep, pos, (int)n, st));
        hipLaunchKernelGGL(user_sets_kernel, G, B, 0, st, n, key_b, keep, pos, ucnt, kuser);
    }
    hipLaunchKernelGGL(widen_kernel, grid_for((uint64_t)n_users + 1), B, 0, st, (uint64_t)n_users + 1, ucnt, uw);
    CF_HIP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tb, uw, uoff, (int)n_users + 1, st));
    // ---- 3-4. co-rated bitmap, row counts, sorted lists ---------------------------------
    CF_HIP_CHECK(ctx, hipMemsetAsync(bm, 0, sizeof(uint32_t) * (size_t)n_movies * words, st));
    if (n_users && n)
        hipLaunchKernelGGL(corated_bits_kernel, dim3(std::min<uint32_t>(n_users, 65536)), dim3(kPrepThreads), 0, st,
                           n_users, uoff, kuser, words, bm);
    CF_HIP_CHECK(ctx, hipMemsetAsync(rcnt, 0, sizeof(uint64_t) * ((uint64_t)n_movies + 1), st));
    if (n_movies) hipLaunchKernelGGL(row_count_kernel, dim3((n_movies + 3) / 4), B, 0, st, n_movies, words, bm, rcnt);
    CF_HIP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tb, rcnt, d_edg_off, (int)n_movies + 1, st));
    if (n_movies)
        hipLaunchKernelGGL(row_write_kernel, dim3(std::min<uint32_t>(n_movies, 65536)), dim3(kPrepThreads), 0, st,
                           n_movies, words, bm, d_edg_off, d_edg_movie, edg_cap);
    CF_HIP_CHECK(ctx, hipGetLastError());
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->prep_ev[1], st));
    return CF_OK;
}

int cf_knn_regroup(cf_ctx* ctx, uint64_t n, uint32_t n_users, uint32_t n_movies, const uint32_t* user,
                   const uint32_t* movie, const float* rating, const uint8_t* validate, uint64_t* train_off,
                   uint32_t* train_user, float* train_rating, uint64_t* test_off, uint32_t* test_user,
                   float* test_rating, uint64_t* edg_off, uint32_t* edg_movie, uint64_t edg_cap) {
    if (!ctx) return CF_EINVAL;
    if ((n && (!user || !movie || !rating || !train_user || !train_rating || !test_user || !test_rating)) ||
        !train_off || !test_off || !edg_off || (edg_cap && !edg_movie))
        return cf_set_error(ctx, CF_EINVAL, "cf_knn_regroup: null argument");
    for (uint64_t i = 0; i < n; ++i)
        if (user[i] >= n_users || movie[i] >= n_movies)
            return cf_set_error(ctx, CF_EINVAL, "cf_knn_regroup: user or movie id out of range");
    CF_TRY(set_device(ctx));
    DevBuf du, dm, dr, dv, dtro, dtru, dtrr, dteo, dteu, dter, deo, dem;
    int rc = CF_OK;
    const size_t off_b = sizeof(uint64_t) * ((size_t)n_movies + 1);
    if (rc == CF_OK) rc = dev_alloc(ctx, du, 4 * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, dm, 4 * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, dr, 4 * n);
    if (rc == CF_OK && validate) rc = dev_alloc(ctx, dv, n);
    if (rc == CF_OK) rc = dev_alloc(ctx, dtro, off_b);
    if (rc == CF_OK) rc = dev_alloc(ctx, dtru, 4 * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, dtrr, 4 * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, dteo, off_b);
    if (rc == CF_OK) rc = dev_alloc(ctx, dteu, 4 * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, dter, 4 * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, deo, off_b);
    if (rc == CF_OK) rc = dev_alloc(ctx, dem, 4 * edg_cap);
    if (rc != CF_OK) return rc;
    if (n) {
        CF_HIP_CHECK(ctx, hipMemcpy(du.p, user, 4 * n, hipMemcpyHostToDevice));
        CF_HIP_CHECK(ctx, hipMemcpy(dm.p, movie, 4 * n, hipMemcpyHostToDevice));
        CF_HIP_CHECK(ctx, hipMemcpy(dr.p, rating, 4 * n, hipMemcpyHostToDevice));
        if (validate) CF_HIP_CHECK(ctx, hipMemcpy(dv.p, validate, n, hipMemcpyHostToDevice));
    }
    CF_TRY(cf_knn_regroup_run(ctx, n, n_users, n_movies, (const uint32_t*)du.p, (const uint32_t*)dm.p,
                              (const float*)dr.p, (const uint8_t*)dv.p, (uint64_t*)dtro.p, (uint32_t*)dtru.p,
                              (float*)dtrr.p, (uint64_t*)dteo.p, (uint32_t*)dteu.p, (float*)dter.p, (uint64_t*)deo.p,
                              (uint32_t*)dem.p, edg_cap, nullptr));
    CF_HIP_CHECK(ctx, hipDeviceSynchronize());
    CF_HIP_CHECK(ctx, hipMemcpy(train_off, dtro.p, off_b, hipMemcpyDeviceToHost));
    CF_HIP_CHECK(ctx, hipMemcpy(test_off, dteo.p, off_b, hipMemcpyDeviceToHost));
    CF_HIP_CHECK(ctx, hipMemcpy(edg_off, deo.p, off_b, hipMemcpyDeviceToHost));
    const uint64_t ntr = train_off[n_movies], nte = test_off[n_movies], ne = edg_off[n_movies];
    if (ntr) {
        CF_HIP_CHECK(ctx, hipMemcpy(train_user, dtru.p, 4 * ntr, hipMemcpyDeviceToHost));
        CF_HIP_CHECK(ctx, hipMemcpy(train_rating, dtrr.p, 4 * ntr, hipMemcpyDeviceToHost));
    }
    if (nte) {
        CF_HIP_CHECK(ctx, hipMemcpy(test_user, dteu.p, 4 * nte, hipMemcpyDeviceToHost));
        CF_HIP_CHECK(ctx, hipMemcpy(test_rating, dter.p, 4 * nte, hipMemcpyDeviceToHost));
    }
    if (std::min(ne, edg_cap)) CF_HIP_CHECK(ctx, hipMemcpy(edg_movie, dem.p, 4 * std::min(ne, edg_cap), hipMemcpyDeviceToHost));
    if (ne > edg_cap)
        return cf_set_error(ctx, CF_ERANGE, "cf_knn_regroup: co-rated lists need " + std::to_string(ne) +
                                                " entries (edg_off[n_movies]); edg_cap is " + std::to_string(edg_cap));
    return CF_OK;
}

int cf_fold_order_run(cf_ctx* ctx, uint64_t n, uint32_t n_users, const uint32_t* d_user, const uint32_t* d_rank,
                      uint32_t* d_order, void* stream_) {
    if (!ctx) return CF_EINVAL;
    if (n >= (1ull << 31)) return cf_set_error(ctx, CF_ERANGE, "cf_fold_order_run: more than 2^31 ratings");
    if (n && (!d_user || !d_rank || !d_order)) return cf_set_error(ctx, CF_EINVAL, "cf_fold_order_run: null argument");
    CF_TRY(set_device(ctx));
    CF_TRY(prep_events(ctx));
    hipStream_t st = (hipStream_t)stream_;
    const int bits_f = bits_for(std::max<uint64_t>(n_users, 1));
    const size_t cub = cub_bytes(n, 1, 64, 64, bits_f, st);
    CF_TRY(prep_reserve(ctx, 3 * 4 * (n + 64) + cub + 1024));
    Carve cv{static_cast<char*>(ctx->d_prep)};
    uint32_t* key_a = cv.take<uint32_t>(n);
    uint32_t* key_b = cv.take<uint32_t>(n);
    uint32_t* idx = cv.take<uint32_t>(n);
    void* tmp = cv.take<char>(cub);
    size_t tb = cub;
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->prep_ev[0], st));
    if (n) {
        hipLaunchKernelGGL(fold_keys_kernel, grid_for(n), dim3(256), 0, st, n, d_user, d_rank, key_a, idx);
        CF_HIP_CHECK(ctx, sort_pairs(tmp, tb, key_a, key_b, idx, d_order, n, bits_f, st));
        CF_HIP_CHECK(ctx, hipGetLastError());
    }
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->prep_ev[1], st));
    return CF_OK;
}

int cf_fold_order(cf_ctx* ctx, uint64_t n, uint32_t n_users, const uint32_t* user, const uint32_t* rank,
                  uint32_t* order) {
    if (!ctx) return CF_EINVAL;
    if (n && (!user || !rank || !order)) return cf_set_error(ctx, CF_EINVAL, "cf_fold_order: null argument");
    std::vector<uint8_t> seen(n_users, 0);
    for (uint32_t u = 0; u < n_users; ++u) {
        if (rank[u] >= n_users || seen[rank[u]]) return cf_set_error(ctx, CF_EINVAL, "cf_fold_order: rank is not a permutation");
        seen[rank[u]] = 1;
    }
    for (uint64_t i = 0; i < n; ++i)
        if (user[i] >= n_users) return cf_set_error(ctx, CF_EINVAL, "cf_fold_order: user id out of range");
    CF_TRY(set_device(ctx));
    DevBuf du, dr, dord;
    int rc = dev_alloc(ctx, du, 4 * n);
    if (rc == CF_OK) rc = dev_alloc(ctx, dr, 4 * (uint64_t)n_users);
    if (rc == CF_OK) rc = dev_alloc(ctx, dord, 4 * n);
    if (rc != CF_OK) return rc;
    if (n) CF_HIP_CHECK(ctx, hipMemcpy(du.p, user, 4 * n, hipMemcpyHostToDevice));
    if (n_users) CF_HIP_CHECK(ctx, hipMemcpy(dr.p, rank, 4 * (uint64_t)n_users, hipMemcpyHostToDevice));
    CF_TRY(cf_fold_order_run(ctx, n, n_users, (const uint32_t*)du.p, (const uint32_t*)dr.p, (uint32_t*)dord.p, nullptr));
    CF_HIP_CHECK(ctx, hipDeviceSynchronize());
    if (n) CF_HIP_CHECK(ctx, hipMemcpy(order, dord.p, 4 * n, hipMemcpyDeviceToHost));
    return CF_OK;
}

int cf_prep_timing(cf_ctx* ctx, float* ms) {
    if (!ctx) return CF_EINVAL;
    if (!ctx->prep_ev[1]) return cf_set_error(ctx, CF_ESTATE, "cf_prep_timing: no prep call yet");
    CF_TRY(set_device(ctx));
    CF_HIP_CHECK(ctx, hipEventSynchronize(ctx->prep_ev[1]));
    float t = 0.0f;
    CF_HIP_CHECK(ctx, hipEventElapsedTime(&t, ctx->prep_ev[0], ctx->prep_ev[1]));
    if (ms) *ms = t;
    return CF_OK;
}
