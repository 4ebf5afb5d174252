// cf_eigen_common.h -- what the LDS Jacobi kernels share (cf_eigen.hip: full matrix in LDS;
// cf_eigen_split.hip: split storage, two users per CU): launch arguments, the 8-lane column-pair
// reductions and the volatile LDS column accesses.  Internal to libcf_mi355x.
#pragma once

#include "cf_internal.h"

namespace cf_eig {

constexpr int kGroup = 8;   // lanes per column pair (half a DPP row)
// Stopping rule: iterate while a sweep made a rotation with |gamma| > kSigRot * tol * sqrt(al be)
// (rotations above tol are always applied).  A numpy model of this kernel on C2 users kept the
// same eigenvalue error and final off-diagonal level with 1-2 fewer sweeps (of ~10) at
// kSigRot = 4..16; on the GPU (C2 mix) 4 / 8 / 16 gave 8.47 / 8.22 / 7.95 sweeps with the same
// parity (profiles/r02/eigen_ab_v4_kappa.txt).  kSigRot2 = kSigRot^2 = 256.
#ifndef CF_EIGEN_SIGROT2
#define CF_EIGEN_SIGROT2 256.0f
#endif
constexpr float kSigRot2 = CF_EIGEN_SIGROT2;

using f2 = __attribute__((ext_vector_type(2))) float;
using f4 = __attribute__((ext_vector_type(4))) float;
// A column read as volatile 8-byte loads: plain loads 64 B apart get fused into
// ds_read2_b64, which the LDS serves at half the rate of two ds_read_b64 (128 vs 256 B/clk;
// MI355X_MICROARCH.md, LDS table).  Volatile accesses are never fused.
__device__ __forceinline__ f2 lds_ld(const f2* p) {
    return *(const volatile __attribute__((address_space(3))) f2*)(p);
}
// Column stores likewise: un-fused ds_write_b64 instead of ds_write2_b64 (CF_EIGEN_FUSED_ST=1
// keeps the compiler's pairing, for A/B).
__device__ __forceinline__ void lds_st(f2* p, f2 v) {
#if defined(CF_EIGEN_FUSED_ST) && CF_EIGEN_FUSED_ST
    *p = v;
#else
    *(volatile __attribute__((address_space(3))) f2*)(p) = v;
#endif
}


template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// All-reduce (sum) over the 8 lanes of a column pair; every lane receives the total.
__device__ __forceinline__ float pair_sum(float x) {
    x += dpp_mov<0xB1>(x);   // quad_perm [1,0,3,2]
    x += dpp_mov<0x4E>(x);   // quad_perm [2,3,0,1]
    x += dpp_mov<0x141>(x);  // row_half_mirror (lanes i <-> 7-i within 8)
    return x;
}

// Launch modes (uniform per launch):
//   kUser  : a2-a4, one user's item subgraph (compute_eigens, precompute_local_threads.cpp)
//   kLocal : a8, one movie's local graph (local_calc.cpp:268-378): star-shaped W, w > 0.1,
//            no 0 -> 1 degree rule, all n eigenpairs, full L2 written out
//   kSigma : a8 w_lim (local_calc.cpp:402-436) of one (movie, test user) pair: the singular
//            values of the unrated rows of the movie's L2, by the same one-sided Jacobi
enum EigenMode : int { kUser = 0, kLocal = 1, kSigma = 2 };

struct EigenArgs {
    int mode;
    const uint32_t* order;
    uint32_t first;
    const uint64_t* item_off;
    const uint32_t* items;
    GraphDev graph;
    uint64_t n_items;
    const uint64_t* evec_off;
    int32_t* m_out;
    float* sigs;
    float* evals;
    float* evecs;
    float tol_scale;
    int max_sweeps;
    // kUser: stop after a sweep with no rotation above stop_rel * sqrt(al be), then one
    // first-order Gram refinement (section 4b) when refine != 0; else the kSigRot * tol rule
    int refine;
    float stop_rel;
    float refine_delta;
    float close_sigrot;   // close pairs converge to close_sigrot * tol
    int sort_sweeps;      // reorder the columns by norm before every sweep: 2 ascending, 1 descending, 0 off
    unsigned long long* stats;
    // kLocal / kSigma
    float* l2;                  // per movie n x n row-major L2 (kLocal writes, kSigma reads)
    const uint64_t* l2_off;
    const uint32_t* pair_movie; // kSigma: unit -> (movie unit, test user)
    const uint32_t* pair_user;
    const uint64_t* test_off;   // test ratings CSR over compact item ids, users ascending
    const uint32_t* test_user;
    const float* test_rating;
    float* wlim;                // kSigma output per pair
    const int* only_flag;       // non-null: run only units j with only_flag[blockIdx.x] != 0
    // kUser, optional: the predictor's complement masks from the gathered W, 3 words per row at
    // 3 * item_off[u] (bit i of word 3r + (i >> 6) = !(w(item_r -> item_i) > 0.1), cf_predict.hip)
    uint64_t* cmask_out;
    uint64_t cmask_words;       // its extent (users beyond it write none)
    uint64_t* cmask_fp;         // per user: cf_items_fp of the items the masks were built from
    uint32_t cmask_users;
    const uint8_t* solved;      // kSigma, spill pairs: w_lim already written (local_wlim_kernel)
    int skip_spill;             // kSigma: every spill pair is solved, no spill launch
    int skip_emax_min;          // > 0: LDS buckets with emax >= it are left out (the hybrid method)
};

// Test rating of `user` for compact item `movie` (0 if absent): binary search of the
// ascending user list (the reference's map lookup with a default of 0, local_calc.cpp:318).
__device__ __forceinline__ float test_rating(const EigenArgs& a, uint32_t movie, uint32_t user) {
    uint64_t lo = a.test_off[movie];
    const uint64_t end = a.test_off[movie + 1];
    uint64_t hi = end;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a.test_user[mid] < user) lo = mid + 1;
        else hi = mid;
    }
    return (lo < end && a.test_user[lo] == user) ? a.test_rating[lo] : 0.0f;
}

// Split-storage Jacobi (cf_eigen_split.hip) for kUser units of the LDS buckets emax >= 9: the
// fixed column of every pair in registers, only the traveling half of B in LDS, so two users share
// a CU.  Kernel A gathers W, assembles B and runs the sweeps, leaving B column-major (ld = k) in the
// user's eigenvector slot and each column's drift d_j in evals[item_off[u] + j]; eigen_kernel's
// RESUME instantiation (cf_eigen.hip) then runs the refinement and the epilogue from there.
// *handled = false (and nothing launched) when the split path does not take this launch.
constexpr int kSplitEmaxMin = 9;    // default smallest bucket of the split layout (cf_set_eigen_split)
constexpr int kSplitEmaxLow = 5;    // smallest bucket it is built for
constexpr int kSplitKmax12 = 180;   // bucket 12: largest k of the split layout (90 LDS slots)
// *finished: the split kernel also ran the refinement and the epilogue (CF_EIGEN_SPLIT_FINISH=1): no
// RESUME launch follows.
int launch_split_sweeps(cf_ctx* ctx, const EigenArgs& a, int emax, uint32_t count, uint32_t kmax, hipStream_t stream,
                        bool* handled, bool* finished);

}  // namespace cf_eig
