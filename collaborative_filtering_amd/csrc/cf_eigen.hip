// cf_eigen.hip -- batched per-user normalized-Laplacian eigendecomposition on gfx950.
//
// Replaces compute_eigens() of precompute_local_threads.cpp:100-213 (same math as
// precompute_local.cpp:165-281).  One workgroup (512 or 1024 threads) owns one user:
//
//   1. gather W_u(i,j) = graph[item_i][item_j] from the HBM-resident dense graph
//      straight into LDS (k x k fp32, column-major, odd leading dimension);
//   2. d_i = row sum (fp64) with the 0 -> 1 rule (:129-141), s_i = sqrt(1/d_i)
//      (:149-153), L2(i,j) = (s_i * L(i,j)) * s_j (:155), sig_min_i from the FULL
//      row (:169-177);
//   3. B = sym_lower(L2) + I in place.  Eigen reads only the lower triangle of L2
//      (:164); the shift makes B positive definite (spectrum of L2 is in [0,2]) so
//      its singular values are its eigenvalues and the rotated columns of B are the
//      eigenvectors scaled by (lambda + 1);
//   4. one-sided (Hestenes) Jacobi sweeps in LDS: each step rotates up to k/2 disjoint
//      column pairs in a recursive-halving ordering that keeps one column of every pair
//      in registers for a whole level (see the loop); a pair is owned by 8 lanes
//      (float2 = ds_read_b64 per row pair, packed v_pk_fma_f32), whose three dot
//      products are reduced with three DPP steps.  Each step reads and writes the
//      whole k x k matrix, so the sweep is bound by LDS bandwidth (128 B/clk/CU),
//      not by VALU issue: 2, 4 and 8 lanes per pair measured 3820, 2828 and 2727
//      cycles per step (tools/probe_eigen.py, 20k users);
//   5. lambda_j = ||b_j|| / ||v_j|| - 1 (||v_j|| tracks the fp32 rotation drift),
//      rank sort ascending, lim (:184-191), write the k x m row-major block, sigs,
//      evals and m.
//
// No MFMA: the matrices are tiny and the work is rotation-shaped, not GEMM-shaped.

#include "cf_eigen_common.h"

namespace {
using namespace cf_eig;

// Bucket geometry: k <= NR = 16 * EMAX rows.  A column is read/written as float2
// (ds_read_b64 / ds_write_b64): lane l of a pair owns rows 16t + 2l, 16t + 2l + 1.
// LD == 16 (mod 64) floats: the 4 consecutive columns that the 4 pairs of a
// half-wave touch in one tournament step start in distinct 16-bank quarters, so the
// b64 accesses are conflict-free (MI355X_MICROARCH.md, LDS table: b64 bank = (a/4) mod 64).
// NARROW (bucket 12 only): at most NC = 188 columns in LDS, so LD = 208 == 16 (mod 64)
// fits too.  The full 192-column bucket falls back to LD = NR + 8 == 8 (mod 64), whose
// b64 column accesses are 2-way bank conflicted; every bucket-12 launch whose largest k
// is <= 188 (all of BASELINE C2/C4: k is clipped at 180) takes the narrow layout.
template <int EMAX, bool NARROW = false>
struct EigenGeom {
    static constexpr int NR = 16 * EMAX;
    static constexpr int NC = NARROW ? 188 : NR;                 // column capacity of B
    static constexpr int E2 = NR / (2 * kGroup);               // float2 chunks per lane
    static constexpr int LD16 = NR + ((16 - NR) % 64 + 64) % 64;
    // == 16 mod 64 where it fits in LDS; the full k <= 192 bucket falls back to NR + 8
    static constexpr int LD = (NC * LD16 + 9 * NR <= 40960 - 4) ? LD16 : NR + 8;
    static constexpr int NT = (NR > 128) ? 1024 : 512;         // 1 pass per step up to NT/8 pairs
    // waves per SIMD the sweeps fit in (their register peak): held for the whole kernel, so
    // the refinement's code cannot push a bucket below it (bucket 5: 6 waves = 3 blocks per CU)
    static constexpr int WPE = EMAX <= 5 ? 6 : 4;   // 3 or 2 blocks of 512 per CU, or 1 of 1024

    static constexpr size_t bytes() {
        return sizeof(float) * (size_t)NC * LD     // B
               + sizeof(uint32_t) * NR             // items
               + sizeof(float) * NR * 5            // s, l2 diagonal, sig, mu, scale drift
               + sizeof(int) * NR                  // perm
               + sizeof(int) * 4;                  // flags
    }
};
static_assert(EigenGeom<12, true>::LD % 64 == 16, "narrow bucket-12 layout must be conflict-free");
static_assert(EigenGeom<12, true>::bytes() <= 163840, "narrow bucket-12 layout exceeds 160 KiB LDS");

// RESUME (kUser, buckets >= kSplitEmaxMin): the split-storage kernel (cf_eigen_split.hip) has run
// stages 1-4 and left B column-major in the user's eigenvector slot, the drifts in evals and the
// sigs written; this instantiation loads them and runs stages 4b and 5.
template <int EMAX, bool NARROW = false, bool RESUME = false>
__global__ __launch_bounds__((EigenGeom<EMAX, NARROW>::NT), (EigenGeom<EMAX, NARROW>::WPE)) void eigen_kernel(EigenArgs a) {
    using G = EigenGeom<EMAX, NARROW>;
    constexpr int NR = G::NR;
    constexpr int LD = G::LD;
    // element (row i, column j) of B.  (A row swizzle for the LD == 8 (mod 64) bucket,
    // to undo its 2-way bank conflicts, measured 12% slower: the modulo costs more.)
    auto bidx = [](int i, int j) { return j * LD + i; };
    constexpr int E2 = G::E2;
    constexpr int NT = G::NT;
    extern __shared__ float smem[];
    float* B = smem;
    uint32_t* s_item = reinterpret_cast<uint32_t*>(B + (size_t)G::NC * LD);
    float* s_s = reinterpret_cast<float*>(s_item + NR);
    float* s_l2d = s_s + NR;
    float* s_sig = s_l2d + NR;
    float* s_mu = s_sig + NR;
    float* s_dev = s_mu + NR;   // d_j = ||v_j||^2 - 1 of the implicit rotation product
    int* s_perm = reinterpret_cast<int*>(s_dev + NR);
    int* s_flag = s_perm + NR;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    constexpr int NW = NT / 64;
    // diagnostics (stats != null): s_memtime per phase, thread 0, summed into stats[4..6]
    unsigned long long t_phase0 = (a.stats && tid == 0) ? __builtin_amdgcn_s_memtime() : 0ull;
    unsigned long long t_phase1 = 0, t_phase2 = 0;
    const int mode = a.mode;
    if (a.only_flag && !a.only_flag[blockIdx.x]) return;
    const uint32_t unit = a.order[a.first + blockIdx.x];
    const uint32_t u = (mode == kSigma) ? a.pair_movie[unit] : unit;   // the graph's unit
    const uint64_t base = a.item_off[u];
    const int nrows = (int)(a.item_off[u + 1] - base);
    int k = nrows;   // columns of B (kSigma: the unrated rows, set below)
    if (nrows <= 0 || nrows > G::NC) {
        if (tid == 0) {
            if (mode == kSigma) a.wlim[unit] = __int_as_float(0x7fc00000);
            else a.m_out[u] = (nrows <= 0) ? 0 : -1;
        }
        return;
    }

    for (int i = tid; i < nrows; i += NT) s_item[i] = a.items[base + i];
    for (int idx = tid; idx < G::NC * LD; idx += NT) B[idx] = 0.0f;
    __syncthreads();
    if constexpr (RESUME) {
        const float* hb = a.evecs + a.evec_off[u];
        // flat over the k x k block, eight loads in flight per thread (a loop per column waited out
        // one HBM round trip per column)
        const int kk = k * k;
#pragma unroll 8
        for (int idx = tid; idx < kk; idx += NT) {
            const int j = idx / k;
            B[bidx(idx - j * k, j)] = hb[idx];
        }
        for (int j = tid; j < k; j += NT) s_dev[j] = a.evals[base + j];
        __syncthreads();
    } else
    if (mode == kSigma) {
        // ---- 1s. B's columns = the unrated rows of the movie's L2 (row 0 counts as
        // unrated, :405-413), in row order (ordered ballot compaction into s_perm)
        const uint32_t user = a.pair_user[unit];
        const bool unr = tid < nrows && (tid == 0 || test_rating(a, s_item[tid], user) == 0.0f);
        const unsigned long long bal = __ballot(unr);
        if (lane == 0) s_perm[NR - 1 - wave] = __popcll(bal);   // per-wave counts (NW <= 16)
        __syncthreads();
        int off = 0;
        for (int w = 0; w < wave; ++w) off += s_perm[NR - 1 - w];
        int h = 0;
        for (int w = 0; w < NW; ++w) h += s_perm[NR - 1 - w];
        __syncthreads();
        if (unr) s_perm[off + __popcll(bal & ((1ull << lane) - 1ull))] = tid;
        __syncthreads();
        k = h;
        const float* L2m = a.l2 + a.l2_off[u];
        for (int c = wave; c < k; c += NW) {
            const float* row = L2m + (size_t)s_perm[c] * nrows;
            for (int j = lane; j < nrows; j += 64) B[bidx(j, c)] = row[j];
        }
        for (int i = tid; i < k; i += NT) s_dev[i] = 0.0f;
        if (tid == 0) s_flag[0] = 0;
        __syncthreads();
    } else {
    // ---- 1. gather W (column-major, B[j*LD + i] = W(i,j)) --------------------------
    // kLocal: W(i, j) = w(item_i -> item_j) if > 0.1 (graph_loader, local_calc.cpp:113);
    // column 0 mirrors row 0: W(i, 0) = w(movie -> item_i) (:331-333); W(0, 0) = 0.
    for (int i = wave; i < k; i += NW) {
        const GraphRow row = a.graph.row(s_item[i]);
        const GraphRow row0 = a.graph.row(s_item[0]);
        for (int j = lane; j < k; j += 64) {
            float w = row[s_item[j]];
            if (mode == kLocal) {
                if (j == 0) w = (i == 0) ? 0.0f : row0[s_item[i]];
                if (!((double)w > 0.1)) w = 0.0f;
            }
            B[bidx(i, j)] = w;
        }
    }
    __syncthreads();
    if (mode == kUser && a.cmask_out && 3 * (base + (uint64_t)k) <= a.cmask_words && u < a.cmask_users) {
        // the predictor's complement masks (local_calc_precomp.cpp:254-265) and the
        // fingerprint of the item list they belong to
        if (wave == 0) {
            const uint64_t fp = cf_items_fp(s_item, k, base, lane);
            if (lane == 0) a.cmask_fp[u] = fp;
        }
        uint64_t* cm = a.cmask_out + 3 * base;
        for (int r = wave; r < k; r += NW)
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const int i = 64 * t + lane;
                const bool out = i < k && !((double)B[bidx(r, min(i, k - 1))] > 0.1);
                const unsigned long long bal = __ballot(out);
                if (lane == 0) cm[3 * r + t] = bal;
            }
    }

    // ---- 2. degrees, D^-1/2, diagonal of L2, sig_min -------------------------------
    for (int i = tid; i < k; i += NT) {
        double d = 0.0;
        for (int j = 0; j < k; ++j) d += (double)B[bidx(i, j)];
        if (d == 0.0 && mode == kUser) d = 1.0;     // (:137-140); local_calc has no guard (:354-360)
        const double s = sqrt(1.0 / d);             // inverse, then sqrt (:149-153)
        s_s[i] = (float)s;
        s_l2d[i] = (float)((s * (d - (double)B[bidx(i, i)])) * s);
    }
    __syncthreads();
    for (int i = tid; i < k; i += NT) {
        const float si = s_s[i];
        float acc = 0.0f;
        for (int j = 0; j < k; ++j) {
            const float l2 = (j == i) ? s_l2d[i] : -(si * B[bidx(i, j)]) * s_s[j];
            acc = fmaf(l2, l2, acc);
        }
        s_sig[i] = sqrtf(acc);                      // (:172-176)
    }
    if (mode == kLocal) {   // the full, unsymmetrised L2 for the w_lim pass (:374, :425-431)
        float* L2m = a.l2 + a.l2_off[u];
        for (int i = wave; i < k; i += NW) {
            const float si = s_s[i];
            for (int j = lane; j < k; j += 64)
                L2m[(size_t)i * k + j] = (j == i) ? s_l2d[i] : -(si * B[bidx(i, j)]) * s_s[j];
        }
    }
    __syncthreads();

    // ---- 3. B = sym_lower(L2) + I, in place ------------------------------------------
    // a wave per column j, lanes down its rows i > j: the lower (i,j) read and write walk
    // a column (conflict-free); only the mirrored (j,i) store strides by LD
    for (int j = wave; j < k; j += NW) {
        const float sj = s_s[j];
        for (int i = j + 1 + lane; i < k; i += 64) {
            const float v = -(s_s[i] * B[bidx(i, j)]) * sj;
            B[bidx(i, j)] = v;   // (i,j), lower
            B[bidx(j, i)] = v;   // (j,i), mirrored
        }
        if (lane == 0) B[bidx(j, j)] = s_l2d[j] + 1.0f;
    }
    for (int i = tid; i < k; i += NT) s_dev[i] = 0.0f;
    if (tid == 0) s_flag[0] = 0;
    __syncthreads();
    }   // mode != kSigma

    if (a.stats && tid == 0) t_phase1 = __builtin_amdgcn_s_memtime();
    // ---- 4. one-sided Jacobi, recursive-halving ordering --------------------------------
    // Level L splits the n columns into 2^L segments (halving each parent, first half
    // rounded up).  In a segment of size s the first f = ceil(s/2) columns are *fixed* --
    // each held by one lane group in registers for the whole level -- and the other
    // s - f *travel*: at step j fixed column i meets traveling column (i + j) mod f.  Every
    // pair of columns meets exactly once per sweep (n - 1 + O(log n) steps), and a step
    // moves one column through LDS instead of two (read, and write back if rotated).
    // Group budget: 2^L * ceil(ceil(n / 2^L) / 2) <= NG for every n <= NR (checked
    // offline for every bucket).
    const int n = (k + 1) & ~1;          // columns incl. the padding column k when k is odd
    const int g = tid / kGroup;
    const int lig = tid % kGroup;
    const float tol = a.tol_scale * sqrtf((float)k) * 2.384185791015625e-07f;  // sqrt(k) * 2^-22
    const float tol2 = tol * tol;
    const bool refine = mode == kUser && a.refine && k > 1;
    // a sweep asks for another one while it made a rotation above this (relative, squared)
    const float stop2 = refine ? a.stop_rel * a.stop_rel : kSigRot2 * tol2;
    // close pairs, |mu_q - mu_p| <~ delta: (be - al)^2 <= 2 delta^2 (al + be) (al, be ~ mu^2)
    const float close2 = refine ? a.close_sigrot * a.close_sigrot * tol2 : stop2;
    const float dclose2 = refine ? 2.0f * a.refine_delta * a.refine_delta : -1.0f;
    // Squared column norms ||b_j||^2 (s_l2d is dead once B is assembled).  A step then
    // needs only the cross product ga = b_p . b_q: the rotated norms follow exactly from
    // (al, be, ga, c, s).  They are recomputed from the columns at every sweep start, and
    // for the fixed columns at every level start, so tracking error stays within a sweep;
    // the eigenvalues (section 5) use fresh fp64 norms.
    float* s_nrm = s_l2d;
    constexpr int NG = NT / kGroup;
    int sweep = 0;
    if constexpr (!RESUME) {
    for (; sweep < a.max_sweeps && k > 1; ++sweep) {
        for (int c = g; c < k; c += NG) {
            const f2* bc = reinterpret_cast<const f2*>(B + c * LD);
            f2 acc = {0.f, 0.f};
#pragma unroll
            for (int e = 0; e < E2; ++e) {
                const f2 x = lds_ld(bc + kGroup * e + lig);
                acc = __builtin_elementwise_fma(x, x, acc);
            }
            const float nc = pair_sum(acc.x + acc.y);
            if (lig == 0) s_nrm[c] = nc;
        }
        __syncthreads();
        if (a.sort_sweeps) {
            // Sorted sweeps (de Rijk's pivoting for one-sided Jacobi): before every sweep the
            // columns move to norm order (ties by index), so the ordering below meets the pairs
            // norm-sorted.  A numpy model of this kernel on C4 users (k 40-180) needed 7.3 instead
            // of 8.1 sweeps for the same eigenvalue error; on the GPU ascending order
            // (the default) took 7.25 sweeps against descending's 7.33, with a lower error.  Column
            // identity means nothing to the result (section 5 ranks by eigenvalue), so this is a
            // relabelling that keeps the sweep's own conflict-free addressing (a slot -> column
            // map read per step instead cost 5% per sweep in bank conflicts and latency).
            // s_perm is free here.
            int* s_map = s_perm;
            const bool asc = a.sort_sweeps == 2;   // ascending order (A/B)
            // rank of column j = #{i : n_i > n_j or (n_i == n_j and i < j)}: a wave per column,
            // the lanes' norms held in registers, three ballots
            {
                constexpr int RB = (NR + 63) / 64;
                float ni[RB];
#pragma unroll
                for (int r = 0; r < RB; ++r) ni[r] = (64 * r + lane < k) ? s_nrm[64 * r + lane] : -1.0f;
                for (int j = wave; j < k; j += NW) {
                    const float nj = s_nrm[j];
                    int rank = 0;
#pragma unroll
                    for (int r = 0; r < RB; ++r) {
                        const int i = 64 * r + lane;
                        const bool before = asc ? ni[r] < nj : ni[r] > nj;
                        rank += __popcll(__ballot(i < k && (before || (ni[r] == nj && i < j))));
                    }
                    if (lane == 0) s_map[rank] = j;
                }
            }
            __syncthreads();
            // the move, 32 rows at a time (<= 4 float2 per thread): every thread loads its part
            // of a row chunk, then stores it once all loads of that chunk are done; the next
            // chunk's loads touch other rows, so one barrier per chunk
            const bool moved = __syncthreads_or(tid < k && s_map[tid] != tid);
            if (moved) {
                constexpr int H = 16;                                // float2 per column chunk
                constexpr int PER = (G::NC * H + NT - 1) / NT;
                const int nf2 = k * H;
                const float dv = tid < k ? s_dev[s_map[tid]] : 0.0f;
                const float nv = tid < k ? s_nrm[s_map[tid]] : 0.0f;
                for (int r0 = 0; r0 < NR / 2; r0 += H) {
                    f2 tmp[PER];
#pragma unroll
                    for (int t = 0; t < PER; ++t) {
                        const int idx = tid + t * NT;
                        const int c = idx >> 4, e = idx & 15;
                        if (idx < nf2 && r0 + e < NR / 2) {
                            tmp[t] = lds_ld(reinterpret_cast<const f2*>(B + s_map[c] * LD) + r0 + e);
                        }
                    }
                    __syncthreads();
#pragma unroll
                    for (int t = 0; t < PER; ++t) {
                        const int idx = tid + t * NT;
                        const int c = idx >> 4, e = idx & 15;
                        if (idx < nf2 && r0 + e < NR / 2) {
                            lds_st(reinterpret_cast<f2*>(B + c * LD) + r0 + e, tmp[t]);
                        }
                    }
                }
                if (tid < k) {
                    s_dev[tid] = dv;
                    s_nrm[tid] = nv;
                }
                __syncthreads();
            }
        }
        for (int L = 0;; ++L) {
            const int segmax = (n + (1 << L) - 1) >> L;
            if (segmax < 2) break;
            const int FL = (segmax + 1) >> 1;   // steps of this level
            const int sigma = g / FL, fi = g - sigma * FL;
            int s0 = 0, s1 = n;
            for (int bit = L - 1; bit >= 0; --bit) {
                const int half = (s1 - s0 + 1) >> 1;
                if ((sigma >> bit) & 1) s0 += half;
                else s1 = s0 + half;
            }
            const int f = (s1 - s0 + 1) >> 1, t = (s1 - s0) - f;
            const int p = s0 + fi;
            const bool fixed = sigma < (1 << L) && fi < f && p < k;
            auto slot = [&](int, int e) { return kGroup * e + lig; };   // float2 of lane lig, chunk e
            f2* bp = reinterpret_cast<f2*>(B + (fixed ? p : 0) * LD);
            f2 xp[E2];
            float devp = 0.0f, al = 0.0f;
            bool pmod = false;
            if (fixed) {
                f2 al2 = {0.f, 0.f};
#pragma unroll
                for (int e = 0; e < E2; ++e) {
                    xp[e] = lds_ld(bp + slot(p, e));
                    al2 = __builtin_elementwise_fma(xp[e], xp[e], al2);
                }
                devp = s_dev[p];
                al = pair_sum(al2.x + al2.y);
            }
            // q = s0 + f + ti walks the traveling half from ti = fi, wrapping at f; a step is
            // live while step < f and the traveling column exists (ti < t, q < k)
            const int tv = fixed ? min(t, k - s0 - f) : 0;
            const int nlive = fixed ? f : 0;
            int ti = fi;
            f2* bq = reinterpret_cast<f2*>(B + (s0 + f + ti) * LD);
            f2* const bq0 = reinterpret_cast<f2*>(B + (s0 + f) * LD);
            for (int step = 0; step < FL; ++step) {
                const int q = s0 + f + ti;
                if (step < nlive && ti < tv) {
                    const float dq = s_dev[q];   // issued with the column loads
                    const float be = s_nrm[q];
                    f2 xq[E2];
                    f2 ga2[2] = {{0.f, 0.f}, {0.f, 0.f}};   // two chains: half the FMA latency
#pragma unroll
                    for (int e = 0; e < E2; ++e) xq[e] = lds_ld(bq + slot(q, e));
#pragma unroll
                    for (int e = 0; e < E2; ++e) ga2[e & 1] = __builtin_elementwise_fma(xp[e], xq[e], ga2[e & 1]);
                    const f2 gs = ga2[0] + ga2[1];
                    const float ga = pair_sum(gs.x + gs.y);
                    if (ga * ga > tol2 * (al * be)) {
                        // Hardware rcp/rsq/sqrt: the rotation only has to annihilate ga well
                        // enough; its scale error (c^2 + s^2 != 1) is tracked exactly below.
                        // t = sign(zeta) / (|zeta| + sqrt(1 + zeta^2)), zeta = (be - al) / (2 ga),
                        // written as 2 ga sign(be - al) / (|be - al| + sqrt((be - al)^2 + 4 ga^2)):
                        // three transcendentals instead of four
                        const float dd = be - al;
                        const float r = __builtin_amdgcn_sqrtf(fmaf(dd, dd, 4.0f * ga * ga));
                        const float tt = (dd < 0.0f ? -2.0f * ga : 2.0f * ga) * __builtin_amdgcn_rcpf(fabsf(dd) + r);
                        const float c = __builtin_amdgcn_rsqf(fmaf(tt, tt, 1.0f));
                        const float sn = c * tt;
                        const f2 c2 = {c, c}, s2 = {sn, sn}, ns2 = {-sn, -sn};
#pragma unroll
                        for (int e = 0; e < E2; ++e) {
                            const f2 np = __builtin_elementwise_fma(ns2, xq[e], c2 * xp[e]);
                            lds_st(bq + slot(q, e), __builtin_elementwise_fma(s2, xp[e], c2 * xq[e]));
                            xp[e] = np;
                        }
                        // c^2 + s^2 = 1 + delta: track each column's accumulated scale so
                        // lambda = ||b_j|| / ||v_j|| - 1 carries no rotation drift.
                        const float delta = fmaf(sn, sn, fmaf(c, c, -1.0f));
                        const float cc = c * c, ss = sn * sn;
                        const float ndp = delta + fmaf(cc, devp, ss * dq);
                        const float csg = 2.0f * c * sn * ga;
                        const float nal = fmaf(cc, al, fmaf(ss, be, -csg));
                        if (lig == 0) {
                            s_dev[q] = delta + fmaf(ss, devp, cc * dq);
                            s_nrm[q] = fmaf(ss, al, fmaf(cc, be, csg));
                            // only a rotation above kSigRot * tol asks for another sweep: the
                            // smaller ones of a sweep leave every pair within tol (their effect
                            // on other pairs is second order) -- the tail sweeps otherwise chase
                            // fp32 rounding noise at the tolerance
                            // with the refinement: pairs closer than refine_delta in mu, which it
                            // leaves alone, still converge to kSigRot * tol
                            const float g2 = ga * ga, ab = al * be, dab = be - al;
                            if (g2 > stop2 * ab || (g2 > close2 * ab && dab * dab <= dclose2 * (al + be)))
                                s_flag[0] = 1;
                        }
                        devp = ndp;
                        al = nal;
                        pmod = true;
                    }
                }
                __syncthreads();
                bq += LD / 2;   // f2 units
                if (++ti == f) {
                    ti = 0;
                    bq = bq0;
                }
            }
            if (pmod) {
#pragma unroll
                for (int e = 0; e < E2; ++e) lds_st(bp + slot(p, e), xp[e]);
                if (lig == 0) {
                    s_dev[p] = devp;
                    s_nrm[p] = al;
                }
            }
            __syncthreads();
        }
        const int rotated = s_flag[0];
        __syncthreads();
        if (!rotated) break;
        if (tid == 0) s_flag[0] = 0;
        __syncthreads();
    }
    }   // !RESUME
    if (a.stats && tid == 0) t_phase2 = __builtin_amdgcn_s_memtime();
    if (!RESUME && a.stats && tid == 0) {
        atomicAdd(&a.stats[0], (unsigned long long)(sweep + 1));
        atomicAdd(&a.stats[1], 1ull);
        atomicMax(&a.stats[2], (unsigned long long)(sweep + 1));
        if (sweep >= a.max_sweeps) atomicAdd(&a.stats[3], 1ull);
    }

    // ---- 4b. first-order Gram refinement (kUser) ---------------------------------------
    // The sweeps stop once no pair rotates by more than stop_rel; what is left is corrected
    // in one step on the matrix cores.  With B = (A + I) V (V's columns orthogonal, norms
    // sqrt(1 + dev)), F = B^T B and mu_j = ||b_j|| / sqrt(1 + dev_j), the eigenvectors are
    // b_j - sum_i b_i K_ij to first order, K_ij = F_ij / (mu_i^2 - mu_j^2) (antisymmetric).
    // Pairs closer than refine_delta in mu are left to the sweeps (first order breaks down
    // there, and a pair inside one eigenvalue cluster changes nothing the predictor reads).
    // V's columns pick up sum_i K_ij^2 of squared norm: dev_j carries it, so the eigenvalues
    // keep their drift-free form.  Wave J owns column tile J: it forms F(:, J) on
    // v_mfma_f32_16x16x4_f32 (exact fp32 FMA chains) -- whose accumulator layout is the B
    // operand layout of the update -- turns it into K(:, J) in registers, and computes
    // B(:, J) - B K(:, J) for every row tile; the new columns are stored once every wave has
    // read B.  (no projector escape at the 1e-2 clustering gap, one sweep fewer.)
    if (refine) {
        for (int c = g; c < k; c += NG) {   // fresh squared norms and mu^2
            const f2* bc = reinterpret_cast<const f2*>(B + c * LD);
            f2 acc = {0.f, 0.f};
#pragma unroll
            for (int e = 0; e < E2; ++e) {
                const f2 x = lds_ld(bc + kGroup * e + lig);
                acc = __builtin_elementwise_fma(x, x, acc);
            }
            const float nc = pair_sum(acc.x + acc.y);
            if (lig == 0) s_mu[c] = nc / (1.0f + s_dev[c]);
        }
        __syncthreads();
        const int nb = (k + 15) >> 4;
        const int m16 = lane & 15, kq = lane >> 4;
        const int j = wave * 16 + m16;   // this lane's column (wave < nb)
        const bool jv = wave < nb && j < k;
        constexpr int HB = (EMAX + 1) / 2;   // row tiles per half
        f4 kv[EMAX];                         // F(:, j), then -K(:, j): the update's B operands
#pragma unroll
        for (int I = 0; I < EMAX; ++I) kv[I] = f4{0.f, 0.f, 0.f, 0.f};
        if (wave < nb) {
            // F(16 I + 4 kq + r, j) for every row tile I: rows 16 c + 4 kq + {0..3} are the
            // k-slots of four MFMAs (the same rows on both operands)
            const f4* pj = reinterpret_cast<const f4*>(B + (jv ? j : 0) * LD + 4 * kq);
            for (int c = 0; c < nb; ++c) {
                const f4 y = jv ? pj[4 * c] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int I0 = 0; I0 < EMAX; I0 += 4) {   // four independent accumulators per group
                    f4 x[4];
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4) {
                        const int ci = (I0 + g4) * 16 + m16;
                        x[g4] = (I0 + g4 < nb && ci < k) ? reinterpret_cast<const f4*>(B + ci * LD + 4 * kq)[4 * c]
                                                         : f4{0.f, 0.f, 0.f, 0.f};
                    }
#pragma unroll
                    for (int t = 0; t < 4; ++t)
#pragma unroll
                        for (int g4 = 0; g4 < 4; ++g4)
                            if (I0 + g4 < EMAX && I0 + g4 < nb)
                                kv[I0 + g4] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[g4][t], y[t], kv[I0 + g4], 0, 0, 0);
                }
            }
            // K(i, j) = F(i, j) / (mu_i^2 - mu_j^2) for i != j, |mu_i - mu_j| > delta; 0 else
            const float muj2 = jv ? s_mu[j] : 1.0f;
            const float muj = sqrtf(muj2);
            const float dlt = a.refine_delta;
            float ksq = 0.0f;
#pragma unroll
            for (int I = 0; I < EMAX; ++I)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = I * 16 + 4 * kq + r;
                    float kvv = 0.0f;
                    if (I < nb && jv && i < k && i != j) {
                        const float mui2 = s_mu[i];
                        if (fabsf(sqrtf(mui2) - muj) > dlt) kvv = kv[I][r] / (mui2 - muj2);
                    }
                    kv[I][r] = -kvv;
                    ksq = fmaf(kvv, kvv, ksq);
                }
            // sum_i K_ij^2 over the four kq quarters (lanes m16 + 16 q): V's column norm growth
            ksq += __shfl_xor(ksq, 16);
            ksq += __shfl_xor(ksq, 32);
            if (kq == 0 && jv) s_dev[j] += ksq;
        }
        // out(R) = B(R, j) + sum_i B(R, i) (-K(i, j)), A operand B(16 R + m16, 16 I + 4 kq + t),
        // in two halves of row tiles: a half's rows are stored after every wave has read them
        // (barrier), and the next half reads only its own rows
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            f4 out[HB];
            if (wave < nb) {
                // HB independent accumulator chains: row tile R = h * HB + q
#pragma unroll
                for (int q = 0; q < HB; ++q) {
                    const int R = h * HB + q;
                    out[q] = (jv && R < nb) ? *reinterpret_cast<const f4*>(B + j * LD + R * 16 + 4 * kq)
                                            : f4{0.f, 0.f, 0.f, 0.f};
                }
#pragma unroll
                for (int I = 0; I < EMAX; ++I) {
                    if (I < nb) {
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int c = I * 16 + 4 * kq + t;
                            const float* bc = B + c * LD + h * HB * 16 + m16;
#pragma unroll
                            for (int q = 0; q < HB; ++q) {
                                if (h * HB + q < nb) {
                                    const float av = c < k ? bc[q * 16] : 0.0f;
                                    out[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, kv[I][t], out[q], 0, 0, 0);
                                }
                            }
                        }
                    }
                }
            }
            __syncthreads();   // every wave has read these rows
            if (jv) {
#pragma unroll
                for (int q = 0; q < HB; ++q) {
                    const int R = h * HB + q;
                    if (R < nb) *reinterpret_cast<f4*>(B + j * LD + R * 16 + 4 * kq) = out[q];
                }
            }
        }
        __syncthreads();
    }

    // ---- 5. eigenvalues, ordering, lim, output ----------------------------------------
    // ||b_j|| accumulated in fp64: a k-term fp32 sum would cost ~k ulps (3e-5 at k=192).
    // Sign convention: sum_i v_ij >= 0.  Eigenvector signs are arbitrary (the reference's
    // come out of Eigen's internals), but the predictor's column filter is signed
    // (local_calc_precomp.cpp:284-304): a fixed convention makes the all-positive
    // lambda = 0 eigenvector of a connected subgraph survive it instead of being dropped
    // from every rating of the user by the luck of the rotation order.
    // One 8-lane group per column in the sweep's float2 layout (conflict-free, rows past
    // nrows are zero), the fp64 partials combined in a fixed butterfly order.
    for (int j = g; j < k; j += NG) {
        const f2* bc = reinterpret_cast<const f2*>(B + j * LD);
        double acc = 0.0, sum = 0.0;
#pragma unroll
        for (int e = 0; e < E2; ++e) {
            const f2 x = lds_ld(bc + kGroup * e + lig);
            acc = fma((double)x.x, (double)x.x, acc);
            acc = fma((double)x.y, (double)x.y, acc);
            sum += (double)x.x;
            sum += (double)x.y;
        }
#pragma unroll
        for (int o = 1; o < kGroup; o <<= 1) {
            acc += __shfl_xor(acc, o);
            sum += __shfl_xor(sum, o);
        }
        if (lig == 0) {
            const double nrm = sqrt(acc);
            s_mu[j] = (float)(nrm / sqrt(1.0 + (double)s_dev[j]));   // lambda_j + 1
            s_s[j] = (float)((sum < 0.0 ? -1.0 : 1.0) / nrm);        // unit-normalises v_j
        }
    }
    __syncthreads();
    if (mode == kSigma) {   // w_lim = sqrt(lambda_min(L2_h L2_h^T)) = sigma_min(L2_h) (:435-436)
        if (tid == 0) {
            float smin = s_mu[0];
            for (int j = 1; j < k; ++j) smin = fminf(smin, s_mu[j]);
            a.wlim[unit] = smin;
        }
        return;
    }
    for (int j = tid; j < k; j += NT) {
        const float mj = s_mu[j];
        int rank = 0;
        for (int i = 0; i < k; ++i) {
            const float mi = s_mu[i];
            rank += (mi < mj) || (mi == mj && i < j);
        }
        s_perm[rank] = j;
    }
    __syncthreads();
    if (mode == kUser) {
        // lim = first sorted position with lambda > smm (:186-188).  lambda = mu - 1 is
        // monotone in mu and the order is ascending in mu, so it equals the count of
        // eigenpairs with !(lambda > smm): one block-wide count instead of a serial walk.
        float smm = 0.0f;
        if constexpr (RESUME) {
            // sigs hold (float)(sig + 0.01), monotone in sig: their max is the max's image
            // (staged through s_sig, which this instantiation does not otherwise use)
            for (int i = tid; i < k; i += NT) s_sig[i] = a.sigs[base + i];
            __syncthreads();
            for (int i = 0; i < k; ++i) smm = fmaxf(smm, s_sig[i]);
        } else {
            for (int i = 0; i < k; ++i)
                if (smm < s_sig[i]) smm = s_sig[i];
            smm = (float)((double)smm + 0.01);          // (:182)
        }
        const bool below = tid < k && !((double)(s_mu[tid] - 1.0f) > (double)smm);
        int lim = __syncthreads_count(below);
        if (lim < 2) lim = 2;                            // (:190-191)
        if (tid == 0) {
            s_flag[1] = lim;
            a.m_out[u] = lim;
        }
    } else if (tid == 0) {
        s_flag[1] = k;   // kLocal keeps every eigenpair (es(ll2), local_calc.cpp:378)
        a.m_out[u] = k;
    }
    __syncthreads();
    const int m = s_flag[1];
    if (mode == kUser && !RESUME)
        for (int i = tid; i < k; i += NT) a.sigs[base + i] = (float)((double)s_sig[i] + 0.01);
    for (int r = tid; r < m && r < k; r += NT) a.evals[base + r] = s_mu[s_perm[r]] - 1.0f;
    if constexpr (RESUME)   // the split kernel's drift scratch past m (the full-LDS kernel leaves it untouched)
        for (int r = m + tid; r < k; r += NT) a.evals[base + r] = 0.0f;
    float* out = a.evecs + a.evec_off[u];
    for (int idx = tid; idx < k * m; idx += NT) {
        const int i = idx / m;
        const int r = idx - i * m;
        float v = 0.0f;
        if (r < k) {
            const int j = s_perm[r];
            v = B[bidx(i, j)] * s_s[j];
        }
        out[idx] = v;
    }
    if (a.stats && tid == 0) {
        const unsigned long long t3 = __builtin_amdgcn_s_memtime();
        atomicAdd(&a.stats[6], t3 - t_phase2);
        if constexpr (!RESUME) {   // the split kernel counts its own phases and steps
            atomicAdd(&a.stats[4], t_phase1 - t_phase0);
            atomicAdd(&a.stats[5], t_phase2 - t_phase1);
            int steps = 0;   // steps per sweep of the recursive-halving ordering
            for (int L = 0; ((n + (1 << L) - 1) >> L) >= 2; ++L) steps += (((n + (1 << L) - 1) >> L) + 1) >> 1;
            atomicAdd(&a.stats[7], (unsigned long long)((sweep + 1) * steps));
        }
    }
}

template <int EMAX, bool NARROW = false, bool RESUME = false>
int launch_bucket_k(cf_ctx* ctx, const EigenArgs& args, uint32_t count, hipStream_t stream) {
    using G = EigenGeom<EMAX, NARROW>;
    const size_t lds = G::bytes();
    static_assert(G::bytes() <= 163840, "eigen bucket exceeds 160 KiB LDS");
    static bool configured = false;
    if (!configured) {
        CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)eigen_kernel<EMAX, NARROW, RESUME>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        configured = true;
    }
    hipLaunchKernelGGL((eigen_kernel<EMAX, NARROW, RESUME>), dim3(count), dim3(G::NT), lds, stream, args);
    CF_HIP_CHECK(ctx, hipGetLastError());
    return CF_OK;
}

// kUser launches of buckets >= kSplitEmaxMin go to the split-storage sweeps (two users per CU)
// followed by the RESUME instantiation (refinement + epilogue) when the split path takes them.
template <int EMAX, bool NARROW = false>
int launch_bucket(cf_ctx* ctx, const EigenArgs& args, uint32_t count, hipStream_t stream, uint32_t kmax = 0) {
    if constexpr (EMAX >= kSplitEmaxLow) {
        bool handled = false, finished = false;
        CF_TRY(launch_split_sweeps(ctx, args, EMAX, count, kmax, stream, &handled, &finished));
        if (handled && finished) return CF_OK;
        if (handled) {
            if (ctx->split_mid_ev) {   // cf_eigen_bucket_timing: the sweeps' share of the bucket
                CF_HIP_CHECK(ctx, hipEventRecord(ctx->split_mid_ev, stream));
                ctx->split_mid_recorded = true;
            }
            return launch_bucket_k<EMAX, NARROW, true>(ctx, args, count, stream);
        }
    }
    return launch_bucket_k<EMAX, NARROW, false>(ctx, args, count, stream);
}

// Bucket 12 in the conflict-free narrow layout when every unit fits it (kmax = the bucket's
// largest k; units are sorted largest first).  CF_EIGEN_NARROW=0 keeps the 192-column layout.
int launch_bucket12_layout(cf_ctx* ctx, const EigenArgs& args, uint32_t count, uint32_t kmax, hipStream_t stream) {
    static const bool narrow_on = [] {
        const char* e = getenv("CF_EIGEN_NARROW");
        return !(e && e[0] == '0');
    }();
    if (narrow_on && kmax <= (uint32_t)EigenGeom<12, true>::NC) return launch_bucket<12, true>(ctx, args, count, stream, kmax);
    return launch_bucket<12>(ctx, args, count, stream, kmax);
}

// kUser: the users above the split layout's largest k (kSplitKmax12; sorted first) take the
// full-LDS kernel in a launch of their own, the rest the split sweeps.
int launch_bucket12(cf_ctx* ctx, const cf_plan* plan, const EigenArgs& args, uint32_t count, uint32_t kmax,
                    hipStream_t stream) {
    if (plan && args.mode == kUser && kmax > (uint32_t)kSplitKmax12 && count > 1) {
        auto k_at = [&](uint32_t j) {
            const uint32_t u = plan->h_order[args.first + j];
            return (uint32_t)(plan->h_item_off[u + 1] - plan->h_item_off[u]);
        };
        uint32_t lo = 0, hi = count;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if (k_at(mid) > (uint32_t)kSplitKmax12) lo = mid + 1;
            else hi = mid;
        }
        if (lo > 0 && lo < count) {
            CF_TRY(launch_bucket12_layout(ctx, args, lo, kmax, stream));
            EigenArgs rest = args;
            rest.first += lo;
            if (rest.only_flag) rest.only_flag += lo;
            return launch_bucket12_layout(ctx, rest, count - lo, k_at(lo), stream);
        }
    }
    return launch_bucket12_layout(ctx, args, count, kmax, stream);
}

}  // namespace

namespace {
// Bucket launches alternate between two context-owned non-blocking streams, forked from and
// joined back to the caller's stream by events: the tail of one bucket (its last users on a
// few CUs) overlaps the start of the next.  Buckets write disjoint users and the kernel keeps
// no global scratch (the spill solver's workspace is per launch and it runs first, alone).
int eigen_fork(cf_ctx* ctx, hipStream_t stream) {
    if (!ctx->aux_stream[0]) {
        for (int i = 0; i < cf_ctx::kAuxStreams; ++i) {
            CF_HIP_CHECK(ctx, hipStreamCreateWithFlags(&ctx->aux_stream[i], hipStreamNonBlocking));
            CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->aux_event[i], hipEventDisableTiming));
        }
        CF_HIP_CHECK(ctx, hipEventCreateWithFlags(&ctx->aux_event[cf_ctx::kAuxStreams], hipEventDisableTiming));
    }
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[cf_ctx::kAuxStreams], stream));
    for (int i = 0; i < cf_ctx::kAuxStreams; ++i) CF_HIP_CHECK(ctx, hipStreamWaitEvent(ctx->aux_stream[i], ctx->aux_event[cf_ctx::kAuxStreams], 0));
    return CF_OK;
}
int eigen_join(cf_ctx* ctx, hipStream_t stream) {
    for (int i = 0; i < cf_ctx::kAuxStreams; ++i) {
        CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[i], ctx->aux_stream[i]));
        CF_HIP_CHECK(ctx, hipStreamWaitEvent(stream, ctx->aux_event[i], 0));
    }
    return CF_OK;
}

int launch_buckets_on(cf_ctx* ctx, const cf_plan* plan, EigenArgs args, hipStream_t caller, bool overlap) {
    hipStream_t stream = caller;
    int nb = 0;
    for (const cf_bucket& b : plan->buckets) {
        if (b.count == 0) continue;
        args.first = b.first;
        if (overlap) {
            // the spill bucket (first) runs alone on stream 0; LDS buckets alternate after it
            if (b.emax == kSpillBucket) {
                stream = ctx->aux_stream[0];
            } else {
                stream = ctx->aux_stream[nb++ % cf_ctx::kAuxStreams];
            }
        }
        int rc;
        if (b.emax == kSpillBucket && args.skip_spill) continue;
        if (args.skip_emax_min > 0 && b.emax >= args.skip_emax_min) continue;
        if (b.emax == kSpillBucket) {
            // n > 192: the fp64 HBM-workspace solver; a8 units in its local-graph / w_lim modes
            cf_spill_local loc{};
            loc.mode = args.mode == kLocal ? 1 : (args.mode == kSigma ? 2 : 0);
            loc.l2 = args.l2;
            loc.l2_off = args.l2_off;
            loc.pair_movie = args.pair_movie;
            loc.pair_user = args.pair_user;
            loc.test_off = args.test_off;
            loc.test_user = args.test_user;
            loc.test_rating = args.test_rating;
            loc.wlim = args.wlim;
            loc.solved = args.solved;
            // overlap: its k > 3072 range keeps running on the spill side stream while the LDS
            // buckets start; launch_all_buckets joins it with the aux streams
            rc = cf_launch_eigen_spill(ctx, plan, b, args.item_off, args.items, args.evec_off, args.m_out, args.sigs,
                                       args.evals, args.evecs, stream, &loc, overlap);
            if (rc != CF_OK) return rc;
            if (overlap) {   // LDS buckets start after the spill solver (it fills every CU)
                CF_HIP_CHECK(ctx, hipEventRecord(ctx->aux_event[0], stream));
                for (int i = 1; i < cf_ctx::kAuxStreams; ++i) CF_HIP_CHECK(ctx, hipStreamWaitEvent(ctx->aux_stream[i], ctx->aux_event[0], 0));
            }
            continue;
        }
        const bool timed = ctx->bucket_timing && args.mode == kUser && b.emax >= 1 && b.emax <= 12;
        const int slot = ctx->bucket_run % cf_ctx::kBucketRuns;
        if (timed) {
            CF_HIP_CHECK(ctx, hipEventRecord(ctx->bucket_ev[slot][b.emax][0], stream));
            ctx->split_mid_ev = ctx->bucket_ev[slot][b.emax][2];
            ctx->split_mid_recorded = false;
        }
        switch (b.emax) {
            case 1: rc = launch_bucket<1>(ctx, args, b.count, stream); break;
            case 2: rc = launch_bucket<2>(ctx, args, b.count, stream); break;
            case 3: rc = launch_bucket<3>(ctx, args, b.count, stream); break;
            case 4: rc = launch_bucket<4>(ctx, args, b.count, stream); break;
            case 5: rc = launch_bucket<5>(ctx, args, b.count, stream, b.kmax); break;
            case 6: rc = launch_bucket<6>(ctx, args, b.count, stream, b.kmax); break;
            case 7: rc = launch_bucket<7>(ctx, args, b.count, stream, b.kmax); break;
            case 8: rc = launch_bucket<8>(ctx, args, b.count, stream, b.kmax); break;
            case 9: rc = launch_bucket<9>(ctx, args, b.count, stream, b.kmax); break;
            case 10: rc = launch_bucket<10>(ctx, args, b.count, stream, b.kmax); break;
            case 11: rc = launch_bucket<11>(ctx, args, b.count, stream, b.kmax); break;
            case 12: rc = launch_bucket12(ctx, plan, args, b.count, b.kmax, stream); break;
            default: return cf_set_error(ctx, CF_ERANGE, "eigen bucket out of range (k > 192)");
        }
        if (rc != CF_OK) return rc;
        if (timed) {
            CF_HIP_CHECK(ctx, hipEventRecord(ctx->bucket_ev[slot][b.emax][1], stream));
            ctx->bucket_recorded[slot][b.emax] = true;
            ctx->bucket_mid[slot][b.emax] = ctx->split_mid_recorded;
            ctx->split_mid_ev = nullptr;
        }
    }
    if (ctx->bucket_timing && args.mode == kUser) ++ctx->bucket_run;
    return CF_OK;
}

int launch_all_buckets(cf_ctx* ctx, const cf_plan* plan, EigenArgs args, hipStream_t caller) {
    const bool overlap = args.mode == kUser && !args.stats;   // diagnostics keep one stream
    if (overlap) CF_TRY(eigen_fork(ctx, caller));
    const int rc = launch_buckets_on(ctx, plan, args, caller, overlap);
    // join on every path: buckets already queued on the aux streams must order before the
    // caller's stream releases or reuses their outputs, also when a later launch failed
    if (overlap) {
        int rj = eigen_join(ctx, caller);
        const int rs = cf_spill_join(ctx, caller);
        if (rj == CF_OK) rj = rs;
        if (rc == CF_OK) return rj;
    }
    return rc;
}
}  // namespace

extern "C" int cf_eigen_bucket_timing_split(cf_ctx* ctx, int enable, float* ms13, float* sweeps_ms13) {
    if (!ctx) return CF_EINVAL;
    CF_TRY(set_device(ctx));
    ctx->split_mid_ev = nullptr;
    if (enable && !ctx->bucket_ev[0][1][0])
        for (auto& run : ctx->bucket_ev)
            for (auto& pr : run)
                for (hipEvent_t& e : pr) CF_HIP_CHECK(ctx, hipEventCreate(&e));
    if (ms13) {   // mean over the recorded runs (the last kBucketRuns of them)
        for (int e = 0; e < 13; ++e) {
            double sum = 0.0, sum_a = 0.0;
            int cnt = 0, cnt_a = 0;
            for (int r = 0; r < cf_ctx::kBucketRuns; ++r) {
                if (!ctx->bucket_recorded[r][e]) continue;
                float ms = 0.0f;
                CF_HIP_CHECK(ctx, hipEventSynchronize(ctx->bucket_ev[r][e][1]));
                CF_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ctx->bucket_ev[r][e][0], ctx->bucket_ev[r][e][1]));
                sum += ms;
                ++cnt;
                if (ctx->bucket_mid[r][e]) {
                    CF_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ctx->bucket_ev[r][e][0], ctx->bucket_ev[r][e][2]));
                    sum_a += ms;
                    ++cnt_a;
                }
                ctx->bucket_recorded[r][e] = false;
                ctx->bucket_mid[r][e] = false;
            }
            ms13[e] = cnt ? (float)(sum / cnt) : -1.0f;
            if (sweeps_ms13) sweeps_ms13[e] = cnt_a ? (float)(sum_a / cnt_a) : -1.0f;
        }
        ctx->bucket_run = 0;
    }
    ctx->bucket_timing = enable != 0;
    return CF_OK;
}

extern "C" int cf_eigen_bucket_timing(cf_ctx* ctx, int enable, float* ms13) {
    return cf_eigen_bucket_timing_split(ctx, enable, ms13, nullptr);
}

int cf_launch_local_eigen(cf_ctx* ctx, const cf_plan* movie_plan, const uint64_t* d_item_off,
                          const uint32_t* d_items, const uint64_t* d_evec_off, float* d_evals,
                          float* d_evecs, float* d_l2, const uint64_t* d_l2_off, int32_t* d_n_out,
                          hipStream_t stream) {
    EigenArgs args{};
    args.mode = kLocal;
    args.order = movie_plan->d_order;
    args.item_off = d_item_off;
    args.items = d_items;
    args.graph = graph_dev(ctx);
    args.n_items = ctx->n_items;
    args.evec_off = d_evec_off;
    args.m_out = d_n_out;
    args.evals = d_evals;
    args.evecs = d_evecs;
    args.l2 = d_l2;
    args.l2_off = d_l2_off;
    args.tol_scale = ctx->tol_scale;
    args.max_sweeps = ctx->max_sweeps;
    args.sort_sweeps = ctx->eigen_sort;
    return launch_all_buckets(ctx, movie_plan, args, stream);
}

int cf_launch_local_sigma(cf_ctx* ctx, const cf_plan* pair_plan, const uint64_t* d_item_off,
                          const uint32_t* d_items, const uint32_t* d_pair_movie,
                          const uint32_t* d_pair_user, const float* d_l2, const uint64_t* d_l2_off,
                          const uint64_t* d_test_off, const uint32_t* d_test_user,
                          const float* d_test_rating, float* d_wlim, hipStream_t stream, const uint8_t* d_solved,
                          bool skip_spill) {
    EigenArgs args{};
    args.mode = kSigma;
    args.solved = d_solved;
    args.skip_spill = skip_spill;
    args.order = pair_plan->d_order;
    args.item_off = d_item_off;
    args.items = d_items;
    args.pair_movie = d_pair_movie;
    args.pair_user = d_pair_user;
    args.l2 = const_cast<float*>(d_l2);
    args.l2_off = d_l2_off;
    args.test_off = d_test_off;
    args.test_user = d_test_user;
    args.test_rating = d_test_rating;
    args.wlim = d_wlim;
    args.tol_scale = ctx->tol_scale;
    args.max_sweeps = ctx->max_sweeps;
    args.sort_sweeps = ctx->eigen_sort;
    return launch_all_buckets(ctx, pair_plan, args, stream);
}

static int launch_emax(cf_ctx* ctx, const cf_plan* plan, int emax, const EigenArgs& args, uint32_t count,
                       uint32_t kmax, hipStream_t stream) {
    switch (emax) {
        case 1: return launch_bucket<1>(ctx, args, count, stream);
        case 2: return launch_bucket<2>(ctx, args, count, stream);
        case 3: return launch_bucket<3>(ctx, args, count, stream);
        case 4: return launch_bucket<4>(ctx, args, count, stream);
        case 5: return launch_bucket<5>(ctx, args, count, stream, kmax);
        case 6: return launch_bucket<6>(ctx, args, count, stream, kmax);
        case 7: return launch_bucket<7>(ctx, args, count, stream, kmax);
        case 8: return launch_bucket<8>(ctx, args, count, stream, kmax);
        case 9: return launch_bucket<9>(ctx, args, count, stream, kmax);
        case 10: return launch_bucket<10>(ctx, args, count, stream, kmax);
        case 11: return launch_bucket<11>(ctx, args, count, stream, kmax);
        case 12: return launch_bucket12(ctx, plan, args, count, kmax, stream);   // the layout cf_launch_eigen picks
        default: return cf_set_error(ctx, CF_ERANGE, "eigen bucket out of range (k > 192)");
    }
}

int cf_launch_eigen_flagged(cf_ctx* ctx, const cf_plan* plan, int emax, uint32_t first, uint32_t count,
                            const int* flag, const uint64_t* d_item_off, const uint32_t* d_items,
                            const uint64_t* d_evec_off, int32_t* d_m, float* d_sigs, float* d_evals,
                            float* d_evecs, hipStream_t stream, uint64_t* d_cmask) {
    if (count == 0) return CF_OK;
    EigenArgs args{};
    args.mode = kUser;
    args.order = plan->d_order;
    args.first = first;
    args.item_off = d_item_off;
    args.items = d_items;
    args.graph = graph_dev(ctx);
    args.n_items = ctx->n_items;
    args.evec_off = d_evec_off;
    args.m_out = d_m;
    args.sigs = d_sigs;
    args.evals = d_evals;
    args.evecs = d_evecs;
    args.tol_scale = ctx->tol_scale;
    args.max_sweeps = ctx->max_sweeps;
    args.sort_sweeps = ctx->eigen_sort;
    args.refine = ctx->eigen_refine;
    args.stop_rel = ctx->stop_rel;
    args.refine_delta = ctx->refine_delta;
    args.close_sigrot = ctx->close_sigrot;
    args.only_flag = flag;
    args.cmask_out = d_cmask;
    args.cmask_words = d_cmask ? ctx->cmask_bytes / sizeof(uint64_t) : 0;
    args.cmask_fp = d_cmask ? ctx->d_cmask_fp : nullptr;
    args.cmask_users = d_cmask ? ctx->cmask_users : 0;
    // units are sorted largest k first within a bucket, so the range's first unit has its kmax
    const uint32_t u0 = plan->h_order[first];
    const uint32_t kmax = (uint32_t)(plan->h_item_off[u0 + 1] - plan->h_item_off[u0]);
    return launch_emax(ctx, plan, emax, args, count, kmax, stream);
}

int cf_launch_eigen(cf_ctx* ctx, const cf_plan* plan, const uint64_t* d_item_off,
                    const uint32_t* d_items, const uint64_t* d_evec_off, int32_t* d_m,
                    float* d_sigs, float* d_evals, float* d_evecs, hipStream_t stream) {
    if (ctx->eigen_method == CF_EIGEN_TRIDIAG) {
        cf_cmask_mark(ctx, plan, d_item_off, d_items, false);
        for (const cf_bucket& b : plan->buckets)
            if (b.emax == kSpillBucket && b.count)
                CF_TRY(cf_launch_eigen_spill(ctx, plan, b, d_item_off, d_items, d_evec_off, d_m, d_sigs, d_evals,
                                             d_evecs, stream));
        return cf_launch_eigen_tri(ctx, plan, d_item_off, d_items, d_evec_off, d_m, d_sigs, d_evals, d_evecs,
                                   stream);
    }
    EigenArgs args{};
    args.mode = kUser;
    args.order = plan->d_order;
    args.item_off = d_item_off;
    args.items = d_items;
    args.graph = graph_dev(ctx);
    args.n_items = ctx->n_items;
    args.evec_off = d_evec_off;
    args.m_out = d_m;
    args.sigs = d_sigs;
    args.evals = d_evals;
    args.evecs = d_evecs;
    args.tol_scale = ctx->tol_scale;
    args.max_sweeps = ctx->max_sweeps;
    args.sort_sweeps = ctx->eigen_sort;
    args.refine = ctx->eigen_refine;
    args.stop_rel = ctx->stop_rel;
    args.refine_delta = ctx->refine_delta;
    args.close_sigrot = ctx->close_sigrot;
    args.stats = ctx->d_stats;
    args.cmask_out = cf_cmask_buffer(ctx, plan);   // the predictor's complement masks
    args.cmask_words = args.cmask_out ? ctx->cmask_bytes / sizeof(uint64_t) : 0;
    args.cmask_fp = args.cmask_out ? ctx->d_cmask_fp : nullptr;
    args.cmask_users = args.cmask_out ? ctx->cmask_users : 0;
    // CF_EIGEN_HYBRID=1 (A/B): bucket 12 (k 177-192) on the Householder + QL path, the other
    // buckets on Jacobi.  Its users get no complement masks (the predictor gathers their rows;
    // their fingerprints stay unwritten, so no stale mask can match)
    static const bool hybrid = [] {
        const char* e = getenv("CF_EIGEN_HYBRID");
        return e && e[0] == '1';
    }();
    bool tri12 = false;
    if (hybrid)
        for (const cf_bucket& b : plan->buckets) tri12 |= b.emax == 12 && b.count > 0;
    if (tri12) {
        args.skip_emax_min = 12;
        if (args.cmask_out && ctx->d_cmask_fp)   // bucket 12 writes none: no fingerprint may survive
            CF_HIP_CHECK(ctx, hipMemsetAsync(ctx->d_cmask_fp, 0, sizeof(uint64_t) * ctx->cmask_users, stream));
    }
    cf_cmask_mark(ctx, plan, d_item_off, d_items, false);
    int rc = launch_all_buckets(ctx, plan, args, stream);
    if (rc == CF_OK && tri12)
        rc = cf_launch_eigen_tri(ctx, plan, d_item_off, d_items, d_evec_off, d_m, d_sigs, d_evals, d_evecs, stream, 12);
    cf_cmask_mark(ctx, plan, d_item_off, d_items, rc == CF_OK && args.cmask_out);
    return rc;
}
