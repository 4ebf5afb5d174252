// cf_knn.hip -- the kNN item-similarity stage on gfx950.
//
// knn2 (knn2.cpp:127-164).  For item pair (a, b) over the users present in both
// train maps (presence, not non-zero: knn.cpp:89-98 loads .predict files with
// rating 0):  num = sum r_a r_b, den1 = sum r_a^2, den2 = sum r_b^2, cnt = #users;
// w = num / (sqrtf(den1) * sqrtf(den2)) if cnt > 5, written when w > 0.01.
// Dense form over the item-major planes R (ratings), S = R*R and B (presence):
//     num = R^T R,  den1 = S^T B,  den2 = B^T S,  cnt = B^T B
// -- four products sharing the same K (user) loop.  Integer ratings in [-11, 11]
// run on v_mfma_i32_32x32x32_i8 (exact; the reference's float accumulators are
// exact too while the sums stay below 2^24), real ratings on
// v_mfma_f32_32x32x2_f32.  The fused epilogue applies the thresholds with IEEE
// sqrtf / division and writes the dense item-weight matrix (the layout the eigen
// stage reads), both directions from one upper-triangle tile.
//
// knn3 (knn3.cpp:185-256), regrouped by user: for each test rating (m, u),
// pred = sum_j w(m,j) r_uj / sum_j w(m,j) over u's test items j with
// w(m, j) > 0.1 (the out-neighbours of m that hold a test rating of u); the squared
// error of round(pred) (0 if pred < 0.1) is accumulated per movie exactly in int64.

#include <algorithm>

#include "cf_internal.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

// ---- plane construction ------------------------------------------------------------
// One thread per (user, rating): item-major planes, [item][user] with leading dim ldu.
__global__ void planes_i8_kernel(uint32_t n_users, const uint64_t* user_off, const uint32_t* item,
                                 const float* rating, uint64_t ldu, int8_t* R, int8_t* S, int8_t* Bp) {
    const uint32_t u = blockIdx.x;
    if (u >= n_users) return;
    for (uint64_t e = user_off[u] + threadIdx.x; e < user_off[u + 1]; e += blockDim.x) {
        const int r = (int)rating[e];
        const size_t idx = (size_t)item[e] * ldu + u;
        R[idx] = (int8_t)r;
        S[idx] = (int8_t)(r * r);
        Bp[idx] = 1;
    }
}

__global__ void planes_f32_kernel(uint32_t n_users, const uint64_t* user_off, const uint32_t* item,
                                  const float* rating, uint64_t ldu, float* R, float* S, float* Bp) {
    const uint32_t u = blockIdx.x;
    if (u >= n_users) return;
    for (uint64_t e = user_off[u] + threadIdx.x; e < user_off[u + 1]; e += blockDim.x) {
        const float r = rating[e];
        const size_t idx = (size_t)item[e] * ldu + u;
        R[idx] = r;
        S[idx] = r * r;
        Bp[idx] = 1.0f;
    }
}

// Upper-triangle tile index -> (ta, tb), ta <= tb.
__device__ __forceinline__ void tile_pair(uint32_t t, uint32_t nt, uint32_t& ta, uint32_t& tb) {
    // rows of decreasing length nt, nt-1, ...: solve with a float estimate, then fix up
    float fn = (float)nt + 0.5f;
    uint32_t a = (uint32_t)(fn - sqrtf(fn * fn - 2.0f * (float)t));
    if (a > 0) --a;
    auto start = [&](uint32_t x) { return x * nt - x * (x - 1) / 2; };
    while (a + 1 < nt && start(a + 1) <= t) ++a;
    while (a > 0 && start(a) > t) --a;
    ta = a;
    tb = a + (t - start(a));
}

struct Knn2Args {
    const void* R;
    const void* S;
    const void* B;
    uint64_t ldu;       // users per plane row (multiple of 32)
    uint32_t n_items;
    uint32_t n_tiles;   // tiles per side (64 items each)
    float w_min;
    int cnt_min;
    float* w_out;       // n_items x n_items
    unsigned int* acc_max;   // max over the diagonal of max(den1, cnt) (float bits), see knn2_store
};

// Epilogue for one 32x32 accumulator block: lane holds column c = lane&31 and rows
// (reg&3) + 8*(reg>>2) + 4*(lane>>5).
template <typename ACC>
__device__ __forceinline__ void knn2_store(const Knn2Args& a, uint32_t a0, uint32_t b0, bool diag_tile,
                                           const ACC& num, const ACC& den1, const ACC& den2,
                                           const ACC& cnt) {
    const int lane = threadIdx.x & 63;
    const uint32_t col = b0 + (lane & 31);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const uint32_t row = a0 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
        if (row >= a.n_items || col >= a.n_items) continue;
        float w = 0.0f;
        if (row != col && (int)cnt[reg] > a.cnt_min) {
            const float fn = (float)num[reg], f1 = (float)den1[reg], f2 = (float)den2[reg];
            const float v = fn / (sqrtf(f1) * sqrtf(f2));                     // (:143)
            if ((double)v > (double)a.w_min) w = v;                           // (:157)
        }
        a.w_out[(size_t)row * a.n_items + col] = w;
        if (!diag_tile) a.w_out[(size_t)col * a.n_items + row] = w;          // w(b,a) == w(a,b)
        // 2^24 guard (SURVEY hard part 7): the diagonal den1 = sum of r^2 over the item's
        // raters bounds every accumulator of every pair through that item (den1, den2
        // directly, |num| by Cauchy-Schwarz, all partial sums included); cnt is counted
        // likewise.  The reference's float accumulators (knn2.cpp:129-140) are exact iff
        // the maximum stays <= 2^24.  One vector atomic per item.
        if (row == col) atomicMax(a.acc_max, __float_as_uint(fmaxf(fabsf((float)den1[reg]), (float)cnt[reg])));
    }
}

// 256 threads = 4 waves; workgroup tile 64 x 64 items, wave (wy, wx) owns 32 x 32.
__global__ __launch_bounds__(256) void knn2_i8_kernel(Knn2Args a) {
    uint32_t ta, tb;
    tile_pair(blockIdx.x, a.n_tiles, ta, tb);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t a0 = ta * 64 + 32 * (wave >> 1), b0 = tb * 64 + 32 * (wave & 1);
    const int r = lane & 31, h = lane >> 5;
    const uint32_t ra = min(a0 + r, a.n_items - 1), rb = min(b0 + r, a.n_items - 1);
    const int8_t* Ra = (const int8_t*)a.R + (size_t)ra * a.ldu + 16 * h;
    const int8_t* Sa = (const int8_t*)a.S + (size_t)ra * a.ldu + 16 * h;
    const int8_t* Ba = (const int8_t*)a.B + (size_t)ra * a.ldu + 16 * h;
    const int8_t* Rb = (const int8_t*)a.R + (size_t)rb * a.ldu + 16 * h;
    const int8_t* Sb = (const int8_t*)a.S + (size_t)rb * a.ldu + 16 * h;
    const int8_t* Bb = (const int8_t*)a.B + (size_t)rb * a.ldu + 16 * h;
    v16i num = {}, den1 = {}, den2 = {}, cnt = {};
    for (uint64_t k0 = 0; k0 < a.ldu; k0 += 32) {
        const v4i ra_ = *(const v4i*)(Ra + k0), sa = *(const v4i*)(Sa + k0), ba = *(const v4i*)(Ba + k0);
        const v4i rb_ = *(const v4i*)(Rb + k0), sb = *(const v4i*)(Sb + k0), bb = *(const v4i*)(Bb + k0);
        num = __builtin_amdgcn_mfma_i32_32x32x32_i8(ra_, rb_, num, 0, 0, 0);
        den1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(sa, bb, den1, 0, 0, 0);
        den2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ba, sb, den2, 0, 0, 0);
        cnt = __builtin_amdgcn_mfma_i32_32x32x32_i8(ba, bb, cnt, 0, 0, 0);
    }
    knn2_store(a, a0, b0, ta == tb, num, den1, den2, cnt);
}

// fp32 planes (real-valued ratings): v_mfma_f32_32x32x2_f32 consumes users
// (s, 16 + s) of each 32-user step as its two k values (h = lane >> 5).
__global__ __launch_bounds__(256) void knn2_f32_kernel(Knn2Args a) {
    uint32_t ta, tb;
    tile_pair(blockIdx.x, a.n_tiles, ta, tb);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t a0 = ta * 64 + 32 * (wave >> 1), b0 = tb * 64 + 32 * (wave & 1);
    const int r = lane & 31, h = lane >> 5;
    const uint32_t ra = min(a0 + r, a.n_items - 1), rb = min(b0 + r, a.n_items - 1);
    const float* Ra = (const float*)a.R + (size_t)ra * a.ldu + 16 * h;
    const float* Sa = (const float*)a.S + (size_t)ra * a.ldu + 16 * h;
    const float* Ba = (const float*)a.B + (size_t)ra * a.ldu + 16 * h;
    const float* Rb = (const float*)a.R + (size_t)rb * a.ldu + 16 * h;
    const float* Sb = (const float*)a.S + (size_t)rb * a.ldu + 16 * h;
    const float* Bb = (const float*)a.B + (size_t)rb * a.ldu + 16 * h;
    v16f num = {}, den1 = {}, den2 = {}, cnt = {};
    for (uint64_t k0 = 0; k0 < a.ldu; k0 += 32) {
#pragma unroll 4
        for (int s = 0; s < 16; ++s) {
            const float xa = Ra[k0 + s], ya = Sa[k0 + s], za = Ba[k0 + s];
            const float xb = Rb[k0 + s], yb = Sb[k0 + s], zb = Bb[k0 + s];
            num = __builtin_amdgcn_mfma_f32_32x32x2f32(xa, xb, num, 0, 0, 0);
            den1 = __builtin_amdgcn_mfma_f32_32x32x2f32(ya, zb, den1, 0, 0, 0);
            den2 = __builtin_amdgcn_mfma_f32_32x32x2f32(za, yb, den2, 0, 0, 0);
            cnt = __builtin_amdgcn_mfma_f32_32x32x2f32(za, zb, cnt, 0, 0, 0);
        }
    }
    knn2_store(a, a0, b0, ta == tb, num, den1, den2, cnt);
}

// ---- knn2 on one code plane ----------------------------------------------------------
// MovieLens-style data has few distinct integer ratings (1..5, plus 0 for .predict
// entries).  With at most 7 distinct values v_1 < ... < v_n, one int8 plane holds
// code = present ? 1 + index(r) : 0 and the three MFMA operands are rebuilt in
// registers with one v_perm_b32 byte lookup per 4 users each:
//     R = tR[code], S = tS[code] = tR[code]^2, B = tB[code] (presence).
// That is a third of the HBM / L2 bytes of the three-plane form.
//
// Tiling: one 512-thread workgroup (8 waves, two per SIMD) per 128 x 128 item tile of
// the upper triangle; wave (wy, wx) owns 64 x 32 = 2 x 1 blocks of 32 x 32, i.e. 8
// int32 accumulators (4 products x 2 blocks, 128 AGPRs).  Users are staged 128 at
// a time through double-buffered LDS (rows padded to 144 B: conflict-free
// ds_read_b128 / ds_write_b128), one barrier per stage.  Per stage a wave issues 32
// MFMAs (1024 SIMD cycles) against 8 KB of staged codes per operand.
//
// Tile order is XCD-aware: 256 consecutive workgroup ids cover a 16 x 16 super-block
// of tiles, and the 32 ids of one XCD (id % 8) a 4 x 8 sub-block, so the tiles that
// run together on one XCD share 12 row bands (1536 items) in its L2.
constexpr int KC_T = 128;            // items per tile side
constexpr int KC_U = 128;            // users per LDS stage
constexpr int KC_ROW = KC_U + 16;    // padded LDS row, bytes

struct Knn2CodeArgs {
    const int8_t* C;
    uint64_t ldu;        // users per plane row (multiple of KC_U)
    uint32_t n_items;
    uint32_t n_tiles;    // tiles per side
    uint32_t n_super;    // super-blocks (16 tiles) per side
    uint32_t tR_lo, tR_hi, tS_lo, tS_hi, tB_lo, tB_hi;   // byte tables, codes 0..3 / 4..7
    float w_min;
    int cnt_min;
    float* w_out;
    unsigned int* acc_max;
    // K-chunk streaming (users beyond one HBM-resident plane): int32 partial sums of the four
    // products per tile, 256 KB per 128 x 128 tile; acc_in: start from them, acc_out: store
    // them instead of running the epilogue (the last chunk has acc_out = 0)
    int* part;
    int acc_in, acc_out;
};

__device__ __forceinline__ bool code_tile(uint32_t b, uint32_t nt, uint32_t nsb, uint32_t& ta, uint32_t& tb) {
    const uint32_t sbi = b >> 8, r = b & 255, x = r & 7, j = r >> 3;
    uint32_t sa, sb;
    tile_pair(sbi, nsb, sa, sb);
    ta = sa * 16 + (x >> 1) * 4 + (j >> 3);
    tb = sb * 16 + (x & 1) * 8 + (j & 7);
    return ta < nt && tb < nt && ta <= tb;
}

__device__ __forceinline__ v4i perm4(uint32_t hi, uint32_t lo, v4i c) {
    v4i o;
    o.x = (int)__builtin_amdgcn_perm(hi, lo, (uint32_t)c.x);
    o.y = (int)__builtin_amdgcn_perm(hi, lo, (uint32_t)c.y);
    o.z = (int)__builtin_amdgcn_perm(hi, lo, (uint32_t)c.z);
    o.w = (int)__builtin_amdgcn_perm(hi, lo, (uint32_t)c.w);
    return o;
}

// 512 threads = 8 waves, two per SIMD: wave (wy, wx) owns 64 x 32 items of the 128 x 128
// tile (2 x 1 blocks of 32 x 32, 8 accumulators = 128 AGPRs), so each SIMD interleaves two
// waves' MFMA streams across LDS-read and barrier latencies.
__global__ __launch_bounds__(512, 1) void knn2_code_kernel(Knn2CodeArgs a) {
    __shared__ __attribute__((aligned(16))) int8_t lds[2][2][KC_T * KC_ROW];   // [buf][A|B], 73,728 B
    uint32_t ta, tb;
    if (!code_tile(blockIdx.x, a.n_tiles, a.n_super, ta, tb)) return;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wy = wave >> 2, wx = wave & 3, r = lane & 31, h = lane >> 5;

    // staging: piece q = t + 512 i (i < KC_P) of each operand is row q / (KC_U / 16), 16-byte
    // segment q % (KC_U / 16)
    constexpr int SEG = KC_U / 16, KC_P = KC_T * SEG / 512, ROWS_PER = 512 / SEG;
    const int8_t* srcA[KC_P];
    const int8_t* srcB[KC_P];
#pragma unroll
    for (int i = 0; i < KC_P; ++i) {
        const uint32_t row = t / SEG + ROWS_PER * i;
        const uint32_t ra = min(ta * KC_T + row, a.n_items - 1), rb = min(tb * KC_T + row, a.n_items - 1);
        srcA[i] = a.C + (size_t)ra * a.ldu + 16 * (t % SEG);
        srcB[i] = a.C + (size_t)rb * a.ldu + 16 * (t % SEG);
    }
    const int st_off = (t / SEG) * KC_ROW + 16 * (t % SEG);   // + ROWS_PER rows per piece
    v4i stA[KC_P], stB[KC_P];
    auto gload = [&](uint64_t k0) {
#pragma unroll
        for (int i = 0; i < KC_P; ++i) {
            stA[i] = *(const v4i*)(srcA[i] + k0);
            stB[i] = *(const v4i*)(srcB[i] + k0);
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < KC_P; ++i) {
            *(v4i*)(&lds[buf][0][st_off + ROWS_PER * i * KC_ROW]) = stA[i];
            *(v4i*)(&lds[buf][1][st_off + ROWS_PER * i * KC_ROW]) = stB[i];
        }
    };

    v16i num[2], den1[2], den2[2], cnt[2];
    // partial-sum slot of this wave: [tile][wave][block i][product][reg][lane] (coalesced per reg)
    const uint64_t tile = (uint64_t)ta * a.n_tiles - (uint64_t)ta * (ta - 1) / 2 + (tb - ta);
    int* part = a.part ? a.part + ((tile * 8 + wave) * 8) * 1024 + lane : nullptr;
    auto part_io = [&](bool load) {
        v16i* acc[4] = {num, den1, den2, cnt};
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    int* q = part + ((i * 4 + p) * 16 + g) * 64;
                    if (load) acc[p][i][g] = *q;
                    else *q = acc[p][i][g];
                }
    };
#pragma unroll
    for (int i = 0; i < 2; ++i) num[i] = den1[i] = den2[i] = cnt[i] = v16i{};
    if (a.acc_in) part_io(true);

    const int rdA = (wy * 64 + r) * KC_ROW + 16 * h, rdB = (wx * 32 + r) * KC_ROW + 16 * h;
    const uint64_t n_stage = a.ldu / KC_U;
    gload(0);
    lstore(0);
    __syncthreads();
    for (uint64_t s = 0; s < n_stage; ++s) {
        const int buf = (int)(s & 1);
        if (s + 1 < n_stage) gload((s + 1) * KC_U);
        const int8_t* LA = lds[buf][0];
        const int8_t* LB = lds[buf][1];
        // codes of k-step ks + 1 are read while the MFMAs of k-step ks issue
        v4i cbn = *(const v4i*)(LB + rdB);
        v4i can[2] = {*(const v4i*)(LA + rdA), *(const v4i*)(LA + rdA + 32 * KC_ROW)};
#pragma unroll
        for (int ks = 0; ks < KC_U / 32; ++ks) {
            const v4i cb = cbn;
            const v4i cac[2] = {can[0], can[1]};
            if (ks + 1 < KC_U / 32) {
                cbn = *(const v4i*)(LB + rdB + 32 * (ks + 1));
                can[0] = *(const v4i*)(LA + rdA + 32 * (ks + 1));
                can[1] = *(const v4i*)(LA + rdA + 32 * KC_ROW + 32 * (ks + 1));
            }
            const v4i Rb = perm4(a.tR_hi, a.tR_lo, cb);
            const v4i Sb = perm4(a.tS_hi, a.tS_lo, cb);
            const v4i Bb = perm4(a.tB_hi, a.tB_lo, cb);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const v4i ca = cac[i];
                const v4i Ra = perm4(a.tR_hi, a.tR_lo, ca);
                const v4i Sa = perm4(a.tS_hi, a.tS_lo, ca);
                const v4i Ba = perm4(a.tB_hi, a.tB_lo, ca);
                num[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Ra, Rb, num[i], 0, 0, 0);
                den1[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Sa, Bb, den1[i], 0, 0, 0);
                den2[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Ba, Sb, den2[i], 0, 0, 0);
                cnt[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Ba, Bb, cnt[i], 0, 0, 0);
            }
        }
        if (s + 1 < n_stage) lstore(buf ^ 1);
        __syncthreads();
    }
    if (a.acc_out) {
        part_io(false);
        return;
    }
    Knn2Args e{};
    e.n_items = a.n_items;
    e.w_min = a.w_min;
    e.cnt_min = a.cnt_min;
    e.w_out = a.w_out;
    e.acc_max = a.acc_max;
    const bool diag = ta == tb;
#pragma unroll
    for (int i = 0; i < 2; ++i)
        knn2_store(e, ta * KC_T + wy * 64 + 32 * i, tb * KC_T + wx * 32, diag, num[i], den1[i], den2[i], cnt[i]);
}

// Which integers in [-11, 11] occur: bit (r + 11) of *mask.
__global__ void rating_mask_kernel(uint64_t n, const float* rating, unsigned int* mask) {
    unsigned int m = 0;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (uint64_t)gridDim.x * blockDim.x)
        m |= 1u << ((int)rating[e] + 11);
    // wave OR-reduce, one atomic per wave
    for (int o = 32; o > 0; o >>= 1) m |= __shfl_xor(m, o);
    if ((threadIdx.x & 63) == 0 && m) atomicOr(mask, m);
}

struct CodeMap {
    int8_t code[23];   // code of rating r at [r + 11]
};

__global__ void plane_code_kernel(uint32_t n_users, const uint64_t* user_off, const uint32_t* item,
                                  const float* rating, uint64_t ldu, CodeMap map, int8_t* C) {
    const uint32_t u = blockIdx.x;
    if (u >= n_users) return;
    for (uint64_t e = user_off[u] + threadIdx.x; e < user_off[u + 1]; e += blockDim.x)
        C[(size_t)item[e] * ldu + u] = map.code[(int)rating[e] + 11];
}

// ---- knn3 ---------------------------------------------------------------------------
struct Knn3Args {
    uint32_t n_users;
    const uint64_t* user_off;
    const uint32_t* items;     // test items of each user (compact ids)
    const float* ratings;      // test ratings
    GraphDev graph;        // dense out_fin_ weights (as parsed floats)
    uint64_t n_items;
    double* pred;              // per test rating, 0 when no neighbour (ratings_knn default)
    unsigned long long* sq_err;  // per movie: sum of tmp^2 (integer-valued for integer ratings)
    double* sq_err_real;       // per movie: same in fp64 (non-integer ratings)
    unsigned int* n_test;      // per movie: number of test ratings
};

__global__ __launch_bounds__(256) void knn3_kernel(Knn3Args a) {
    const uint32_t u = blockIdx.x;
    if (u >= a.n_users) return;
    const uint64_t base = a.user_off[u];
    const int k = (int)(a.user_off[u + 1] - base);
    for (int r = threadIdx.x; r < k; r += blockDim.x) {
        const uint32_t m = a.items[base + r];
        const GraphRow wrow = a.graph.row(m);
        double sw = 0.0, swr = 0.0;
        for (int j = 0; j < k; ++j) {
            const float w = wrow[a.items[base + j]];
            if ((double)w > 0.1) {                               // knn3.cpp:91
                sw += (double)w;
                swr += (double)w * (double)a.ratings[base + j];  // :202
            }
        }
        const double pred = sw > 0.0 ? swr / sw : 0.0;           // :216, missing key -> 0
        a.pred[base + r] = pred;
        const float tmp = (pred < 0.1) ? 0.0f : (float)((double)a.ratings[base + r] - round(pred));  // :243-246
        const float sq = tmp * tmp;
        atomicAdd(&a.sq_err[m], (unsigned long long)sq);
        atomicAdd(&a.sq_err_real[m], (double)sq);
        atomicAdd(&a.n_test[m], 1u);
    }
}

}  // namespace

static int knn2_alloc(cf_ctx* ctx, size_t need) {
    if (need > ctx->knn_bytes) {
        if (ctx->d_knn) (void)hipFree(ctx->d_knn);
        ctx->d_knn = nullptr;
        ctx->knn_bytes = 0;
        if (hipMalloc(&ctx->d_knn, need) != hipSuccess)
            return cf_set_error(ctx, CF_ENOMEM, "knn2 planes (" + std::to_string(need) + " bytes)");
        ctx->knn_bytes = need;
    }
    return CF_OK;
}

// Byte tables of the code path: codes 0..7 -> value, packed as two little-endian dwords.
static void code_tables(const int* vals, int n, uint32_t& rlo, uint32_t& rhi, uint32_t& slo, uint32_t& shi,
                        uint32_t& blo, uint32_t& bhi) {
    uint8_t R[8] = {}, S[8] = {}, B[8] = {};
    for (int c = 1; c <= n; ++c) {
        R[c] = (uint8_t)(int8_t)vals[c - 1];
        S[c] = (uint8_t)(vals[c - 1] * vals[c - 1]);
        B[c] = 1;
    }
    auto pack = [](const uint8_t* b) { return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24; };
    rlo = pack(R), rhi = pack(R + 4), slo = pack(S), shi = pack(S + 4), blo = pack(B), bhi = pack(B + 4);
}

int cf_launch_knn2(cf_ctx* ctx, uint32_t n_users, uint32_t n_items, const uint64_t* d_user_off,
                   const uint32_t* d_item, const float* d_rating, int integer_ratings, float w_min,
                   int cnt_min, float* d_w_out, hipStream_t stream) {
    if (n_items == 0) return CF_OK;
    for (hipEvent_t& e : ctx->knn_ev)
        if (!e) CF_HIP_CHECK(ctx, hipEventCreate(&e));
    if (!ctx->d_knn_acc) CF_HIP_CHECK(ctx, hipMalloc(&ctx->d_knn_acc, sizeof(unsigned int)));
    CF_HIP_CHECK(ctx, hipMemsetAsync(ctx->d_knn_acc, 0, sizeof(unsigned int), stream));
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->knn_ev[0], stream));
    // Integer ratings: which values occur decides between one code plane (<= 7 values)
    // and the three-plane int8 form.  The scan reads the ratings once (n x 4 B).
    int vals[23], n_vals = 99;
    if (integer_ratings) {
        uint64_t n_rat = 0;
        CF_HIP_CHECK(ctx, hipMemcpyAsync(&n_rat, d_user_off + n_users, sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
        CF_TRY(knn2_alloc(ctx, 16));
        unsigned int* d_mask = (unsigned int*)ctx->d_knn;
        CF_HIP_CHECK(ctx, hipMemsetAsync(d_mask, 0, sizeof(unsigned int), stream));
        CF_HIP_CHECK(ctx, hipStreamSynchronize(stream));
        if (n_rat) {
            const uint32_t grid = (uint32_t)std::min<uint64_t>((n_rat + 255) / 256, 4096);
            hipLaunchKernelGGL(rating_mask_kernel, dim3(grid), dim3(256), 0, stream, n_rat, d_rating, d_mask);
            CF_HIP_CHECK(ctx, hipGetLastError());
        }
        unsigned int mask = 0;
        CF_HIP_CHECK(ctx, hipMemcpyAsync(&mask, d_mask, sizeof(mask), hipMemcpyDeviceToHost, stream));
        CF_HIP_CHECK(ctx, hipStreamSynchronize(stream));
        n_vals = 0;
        for (int b = 0; b < 23; ++b)
            if (mask >> b & 1) vals[n_vals++] = b - 11;
    }
    if (integer_ratings && n_vals <= 7) {
        // Users in K chunks when one code plane of every user would not fit (SURVEY 8f item 3:
        // 1M x 50k is a 50 GB plane; the int32 partials are 256 KB per tile, 20 GB at 50k
        // items): a plane per chunk, partial sums carried across chunks in HBM, the epilogue
        // on the last chunk.  cf_set_knn2_chunk forces a chunk size (tests).
        const uint64_t n_tiles = (n_items + KC_T - 1) / KC_T;
        const uint64_t ldu_all = ((uint64_t)n_users + KC_U - 1) / KC_U * KC_U;
        uint64_t chunk = ldu_all;
        if (ctx->knn_chunk_users) {
            chunk = std::max<uint64_t>(KC_U, (uint64_t)ctx->knn_chunk_users / KC_U * KC_U);
        } else {
            size_t free_b = 0, total_b = 0;
            CF_HIP_CHECK(ctx, hipMemGetInfo(&free_b, &total_b));
            const size_t avail = (free_b + ctx->knn_bytes) / 10 * 6;   // leave room for the caller
            if ((size_t)n_items * ldu_all > avail) {
                const size_t parts = n_tiles * (n_tiles + 1) / 2 * 262144;
                if (parts >= avail) return cf_set_error(ctx, CF_ENOMEM, "knn2: tile partial sums exceed HBM");
                chunk = std::max<uint64_t>(KC_U, (avail - parts) / n_items / KC_U * KC_U);
            }
        }
        chunk = std::min(chunk, ldu_all);
        const uint64_t n_chunks = n_users ? (n_users + chunk - 1) / chunk : 1;
        const size_t plane = (size_t)n_items * chunk;
        CF_TRY(knn2_alloc(ctx, std::max<size_t>(plane, 16)));
        int8_t* C = (int8_t*)ctx->d_knn;
        int* part = nullptr;
        if (n_chunks > 1) {
            const size_t pb = n_tiles * (n_tiles + 1) / 2 * 262144;
            if (pb > ctx->knn_part_bytes) {
                if (ctx->d_knn_part) (void)hipFree(ctx->d_knn_part);
                ctx->d_knn_part = nullptr;
                ctx->knn_part_bytes = 0;
                if (hipMalloc(&ctx->d_knn_part, pb) != hipSuccess)
                    return cf_set_error(ctx, CF_ENOMEM, "knn2 tile partial sums (" + std::to_string(pb) + " bytes)");
                ctx->knn_part_bytes = pb;
            }
            part = (int*)ctx->d_knn_part;
        }
        CodeMap map{};
        for (int c = 1; c <= n_vals; ++c) map.code[vals[c - 1] + 11] = (int8_t)c;
        Knn2CodeArgs a{};
        a.C = C;
        a.ldu = chunk;
        a.n_items = n_items;
        a.n_tiles = (uint32_t)n_tiles;
        a.n_super = (a.n_tiles + 15) / 16;
        code_tables(vals, n_vals, a.tR_lo, a.tR_hi, a.tS_lo, a.tS_hi, a.tB_lo, a.tB_hi);
        a.w_min = w_min;
        a.cnt_min = cnt_min;
        a.w_out = d_w_out;
        a.acc_max = ctx->d_knn_acc;
        a.part = part;
        const uint32_t grid = a.n_super * (a.n_super + 1) / 2 * 256;
        ctx->knn_path = 1;
        ctx->knn_chunks = (int)n_chunks;
        for (uint64_t c = 0; c < n_chunks; ++c) {
            const uint64_t u0 = c * chunk;
            const uint32_t nu = (uint32_t)std::min<uint64_t>(chunk, n_users - std::min<uint64_t>(u0, n_users));
            CF_HIP_CHECK(ctx, hipMemsetAsync(C, 0, plane, stream));
            if (nu) {
                hipLaunchKernelGGL(plane_code_kernel, dim3(nu), dim3(64), 0, stream, nu, d_user_off + u0, d_item,
                                   d_rating, chunk, map, C);
                CF_HIP_CHECK(ctx, hipGetLastError());
            }
            a.acc_in = c > 0;
            a.acc_out = c + 1 < n_chunks;
            if (c == 0) CF_HIP_CHECK(ctx, hipEventRecord(ctx->knn_ev[1], stream));
            hipLaunchKernelGGL(knn2_code_kernel, dim3(grid), dim3(512), 0, stream, a);
            CF_HIP_CHECK(ctx, hipGetLastError());
        }
        CF_HIP_CHECK(ctx, hipEventRecord(ctx->knn_ev[2], stream));
        return CF_OK;
    }
    ctx->knn_chunks = 1;
    const uint64_t ldu = ((uint64_t)n_users + 31) / 32 * 32;
    const size_t esz = integer_ratings ? 1 : 4;
    const size_t plane = (size_t)n_items * ldu * esz;
    const size_t need = 3 * plane;
    CF_TRY(knn2_alloc(ctx, need));
    char* base = (char*)ctx->d_knn;
    CF_HIP_CHECK(ctx, hipMemsetAsync(base, 0, need, stream));
    if (n_users) {
        if (integer_ratings)
            hipLaunchKernelGGL(planes_i8_kernel, dim3(n_users), dim3(64), 0, stream, n_users, d_user_off, d_item,
                               d_rating, ldu, (int8_t*)base, (int8_t*)(base + plane), (int8_t*)(base + 2 * plane));
        else
            hipLaunchKernelGGL(planes_f32_kernel, dim3(n_users), dim3(64), 0, stream, n_users, d_user_off, d_item,
                               d_rating, ldu, (float*)base, (float*)(base + plane), (float*)(base + 2 * plane));
        CF_HIP_CHECK(ctx, hipGetLastError());
    }
    Knn2Args a{};
    a.R = base;
    a.S = base + plane;
    a.B = base + 2 * plane;
    a.ldu = ldu;
    a.n_items = n_items;
    a.n_tiles = (n_items + 63) / 64;
    a.w_min = w_min;
    a.cnt_min = cnt_min;
    a.w_out = d_w_out;
    a.acc_max = ctx->d_knn_acc;
    const uint32_t ntp = a.n_tiles * (a.n_tiles + 1) / 2;
    ctx->knn_path = integer_ratings ? 2 : 3;
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->knn_ev[1], stream));
    if (ntp) {
        if (integer_ratings)
            hipLaunchKernelGGL(knn2_i8_kernel, dim3(ntp), dim3(256), 0, stream, a);
        else
            hipLaunchKernelGGL(knn2_f32_kernel, dim3(ntp), dim3(256), 0, stream, a);
        CF_HIP_CHECK(ctx, hipGetLastError());
    }
    CF_HIP_CHECK(ctx, hipEventRecord(ctx->knn_ev[2], stream));
    return CF_OK;
}

int cf_launch_knn3(cf_ctx* ctx, uint32_t n_users, const uint64_t* d_user_off, const uint32_t* d_items,
                   const float* d_ratings, double* d_pred, unsigned long long* d_sq, double* d_sq_real,
                   unsigned int* d_cnt, hipStream_t stream) {
    Knn3Args a{};
    a.n_users = n_users;
    a.user_off = d_user_off;
    a.items = d_items;
    a.ratings = d_ratings;
    a.graph = graph_dev(ctx);
    a.n_items = ctx->n_items;
    a.pred = d_pred;
    a.sq_err = d_sq;
    a.sq_err_real = d_sq_real;
    a.n_test = d_cnt;
    if (n_users) {
        hipLaunchKernelGGL(knn3_kernel, dim3(n_users), dim3(256), 0, stream, a);
        CF_HIP_CHECK(ctx, hipGetLastError());
    }
    return CF_OK;
}
