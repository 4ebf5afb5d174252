// cf_eigen_split.hip -- the Jacobi sweeps of compute_eigens (precompute_local_threads.cpp:164-166)
// for users with 128 < k <= 180 in a split layout that lets two users share a CU.
//
// cf_eigen.hip keeps the whole k x k matrix B in LDS: 130 KB at k = 180, so one user holds a CU
// and its step -- LDS reads, the dot product, the rotation, the LDS writes, a barrier -- leaves the
// LDS idle while the VALU works and the other way round (one user per CU at k = 180
// takes 5.2 us per user, the same step with two users per CU 3.8 us).  Here only the traveling
// half of the recursive-halving ordering lives in LDS (k/2 column slots, <= 80 KB); the fixed
// column of every pair stays in the registers of its 8-lane group for the whole level, and from
// one level to the next only the columns that change role move, by swaps (a group writes its
// column into the slot it reads its next one from).  The schedule of those moves depends only on
// k; it is built and verified on the host once (build_schedule / verify_schedule) and read from a
// small table by the kernel.
//
// Kernel A (split_sweep_kernel, one workgroup per user, two per CU):
//   1. gather W_u from the graph into the user's eigenvector slot (row-major, k x k; the slot
//      holds k * max(k, 2) floats), with the predictor's complement masks;
//   2. degrees (fp64, the 0 -> 1 rule), s = sqrt(1/d), the L2 diagonal and sig_min from the full
//      rows -- the same arithmetic, in the same order, as cf_eigen.hip stage 2;
//   3. B = sym_lower(L2) + I assembled in place, 64 columns at a time through LDS (the slot ends up
//      column-major, column c at c * k), with the columns' norms;
//   4. sweeps: each one loads its columns from the slot in norm order (the sorted sweeps of
//      cf_eigen.hip), fixed half into registers and traveling half into LDS, runs the levels, and
//      writes every column back with its fresh norm and drift; the sweep's stop rule is
//      cf_eigen.hip's;
//   5. the drift of every column to evals[item_off[u] + j].
// eigen_kernel<EMAX, NARROW, true> (cf_eigen.hip) then loads B and the drifts into its full LDS
// layout and runs the Gram refinement and the epilogue unchanged.

#include <array>
#include <mutex>

#include "cf_eigen_common.h"

namespace cf_eig {
namespace {

constexpr int kMaxLev = 9;          // levels of the recursive halving for k <= 256
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kRoleActive = 1u << 31;
constexpr uint32_t kTrWrite = 1u << 31;
constexpr uint32_t kTrRead = 1u << 30;

constexpr int split_ld(int nr) {   // smallest LD >= nr with LD == 16 or 48 (mod 64): conflict-free
    int ld = nr;
    while (ld % 64 != 16 && ld % 64 != 48) ++ld;
    return ld;
}

// users per CU by bucket: LDS (<= 160 KB / UPC) and the sweeps' registers (512 / ceil(UPC * EMAX / 4)
// per lane, 4 * EMAX for the two columns of a pair plus ~30) both have to fit
constexpr int split_upc(int emax) { return emax >= 9 ? 2 : 3; }

template <int EMAX>
struct SplitGeom {
    static constexpr int NR = 16 * EMAX;                  // rows (zero past k)
    static constexpr int E2 = EMAX;                       // float2 per lane: rows 16e + 2lig, +1
    static constexpr int NG = 8 * EMAX;                   // lane groups
    static constexpr int NT = kGroup * NG;
    static constexpr int NS = EMAX == 12 ? 90 : 8 * EMAX;   // LDS column slots
    static constexpr int KLO = 16 * (EMAX - 1) + 1;
    static constexpr int KHI = EMAX == 12 ? kSplitKmax12 : NR;   // largest k the layout takes
    static constexpr int LD = split_ld(NR);
    static constexpr int UPC = split_upc(EMAX);           // users per CU
    // waves per SIMD the registers are sized for: a workgroup's EMAX waves land on the SIMDs
    // round-robin from a varying start, so UPC of them may stack ceil(EMAX / 4) each on one SIMD
    static constexpr int WPE = UPC * ((EMAX + 3) / 4);
    // assembly: columns per LDS tile (the tile lives in the slot area)
    static constexpr int CB = (NS * LD) / (KHI + 1) < 64 ? (NS * LD) / (KHI + 1) : 64;
    // table words per k: nlev, f0, FL[kMaxLev], role[kMaxLev][NG], trans[kMaxLev][NG], end_g[NG], end_s[NS]
    static constexpr int OFF_FL = 2;
    static constexpr int OFF_ROLE = OFF_FL + kMaxLev;
    static constexpr int OFF_TR = OFF_ROLE + kMaxLev * NG;
    static constexpr int OFF_ENDG = OFF_TR + kMaxLev * NG;
    static constexpr int OFF_ENDS = OFF_ENDG + NG;
    static constexpr int STRIDE = OFF_ENDS + NS;
    static constexpr size_t bytes() {
        return sizeof(float) * ((size_t)NS * LD   // traveling slots (the assembly's tile before)
                                + 2 * NS          // tracked norm, drift per slot
                                + 4 * NR)         // fresh norm, drift per column; s; L2 diagonal
               + sizeof(uint32_t) * NR            // items
               + sizeof(int) * NR                 // rank -> column
               + sizeof(int) * 4                  // flags
               + sizeof(unsigned long long) * 3;  // phase stamps (cf_debug_stats)
    }
    static_assert(bytes() * UPC <= 163840, "UPC users must share a CU's LDS");
    static_assert(WPE <= 8, "at most 8 waves per SIMD");
    static_assert(CB >= 16, "assembly tile");
};

// ------------------------------------------------------------------------------------------------
// Host: the schedule.  Level L splits every segment of >= 2 columns into a fixed part F (in lane
// groups) and a traveling part T (in consecutive LDS slots); fixed F[i] meets T[(i + j) mod P] at
// step j < P = max(|F|, |T|).  Odd segments are split ceil or floor so that neither the groups nor
// the slots overflow (the plain ceil split holds ~2k/3 fixed columns at the deep levels).
struct Seg {
    std::vector<int> cols;
    int f;   // fixed count (1 for a lone column)
};

struct Schedule {
    int n = 0, f0 = 0, nlev = 0;
    int FL[kMaxLev] = {};
    std::vector<uint32_t> role, trans;   // [kMaxLev][NG]
    std::vector<uint32_t> end_g, end_s;  // column label held at the end of the sweep
    std::vector<std::vector<Seg>> segs;  // per level (for verification)
    int max_groups = 0, max_slots = 0;
};

bool build_schedule(int n, int NG, int NS, Schedule& S) {
    S = Schedule{};
    S.n = n;
    S.role.assign((size_t)kMaxLev * NG, 0u);
    S.trans.assign((size_t)kMaxLev * NG, 0u);
    if (n < 2) return false;
    const int f0 = (n + 1) / 2;
    if (f0 > NG || n - f0 > NS) return false;
    S.f0 = f0;
    std::vector<int> reg(n, -1), slot(n, -1);   // column -> group / slot
    for (int c = 0; c < f0; ++c) reg[c] = c;
    for (int x = 0; x < n - f0; ++x) slot[f0 + x] = x;
    std::vector<Seg> segs{Seg{{}, f0}};
    for (int c = 0; c < n; ++c) segs[0].cols.push_back(c);
    for (int L = 0;; ++L) {
        bool any = false;
        for (const Seg& s : segs) any |= s.cols.size() >= 2;
        if (!any) break;
        if (L >= kMaxLev) return false;
        // ---- the level's roles
        int FL = 0, ng = 0, ns = 0;
        for (const Seg& s : segs) {
            if (s.cols.size() < 2) continue;
            const int f = s.f, t = (int)s.cols.size() - f, P = std::max(f, t);
            FL = std::max(FL, P);
            const int base = t ? slot[s.cols[f]] : 0;
            for (int x = 0; x < t; ++x)
                if (slot[s.cols[f + x]] != base + x) return false;   // traveling slots consecutive
            for (int i = 0; i < f; ++i) {
                const int g = reg[s.cols[i]];
                if (g < 0) return false;
                S.role[(size_t)L * NG + g] = kRoleActive | (uint32_t)i | ((uint32_t)P << 8) | ((uint32_t)t << 16) |
                                              ((uint32_t)base << 24);
            }
        }
        for (int c = 0; c < n; ++c) {
            ng += reg[c] >= 0;
            ns += slot[c] >= 0;
        }
        S.max_groups = std::max(S.max_groups, ng);
        S.max_slots = std::max(S.max_slots, ns);
        S.FL[L] = FL;
        S.segs.push_back(segs);
        S.nlev = L + 1;
        // ---- the transition to level L + 1: children F and T of every live segment
        struct Child {
            std::vector<int> F, T;
            bool lone;
        };
        std::vector<Child> ch;
        for (const Seg& s : segs) {
            if (s.cols.size() >= 2)
                ch.push_back({std::vector<int>(s.cols.begin(), s.cols.begin() + s.f),
                              std::vector<int>(s.cols.begin() + s.f, s.cols.end()), false});
            else
                ch.push_back({s.cols, {}, true});
        }
        std::vector<char> gused(NG, 0), sused(NS, 0);
        for (int c = 0; c < n; ++c) {
            if (reg[c] >= 0) gused[reg[c]] = 1;
            if (slot[c] >= 0) sused[slot[c]] = 1;
        }
        std::vector<int> free_g, free_s;
        for (int g = 0; g < NG; ++g)
            if (!gused[g]) free_g.push_back(g);
        for (int x = 0; x < NS; ++x)
            if (!sused[x]) free_s.push_back(x);
        auto opts_of = [](int size) {
            std::vector<int> o{(size + 1) / 2};
            if (size / 2 != (size + 1) / 2) o.push_back(size / 2);
            return o;
        };
        // per parent: options (fF, fT); nout / nin as functions of the choice
        std::vector<std::vector<std::pair<int, int>>> plans(ch.size());
        auto nout_of = [&](const Child& c, int fF) { return c.F.size() >= 2 ? (int)c.F.size() - fF : 0; };
        auto nin_of = [&](const Child& c, int fT) { return c.T.size() >= 2 ? fT : 0; };
        for (size_t p = 0; p < ch.size(); ++p) {
            const Child& c = ch[p];
            if (c.lone) {
                plans[p].push_back({1, 0});
                continue;
            }
            const std::vector<int> fFs = c.F.size() >= 2 ? opts_of((int)c.F.size()) : std::vector<int>{(int)c.F.size()};
            const std::vector<int> fTs = c.T.size() >= 2 ? opts_of((int)c.T.size()) : std::vector<int>{(int)c.T.size()};
            for (int fF : fFs)
                for (int fT : fTs) {
                    const int no = nout_of(c, fF), ni = nin_of(c, fT);
                    if (no > ni && !(no == 1 && ni == 0)) continue;   // the F-child's travelers take the in-slots
                    plans[p].push_back({fF, fT});
                }
            if (plans[p].empty()) return false;
        }
        std::vector<std::pair<int, int>> choice(ch.size());
        for (size_t p = 0; p < ch.size(); ++p) choice[p] = plans[p][0];
        // columns lone after the transition (never moved by swaps; may be parked)
        std::vector<int> lone_all;
        for (const Child& c : ch) {
            if (c.lone) {
                lone_all.push_back(c.F[0]);
                continue;
            }
            if (c.F.size() == 1) lone_all.push_back(c.F[0]);
            if (c.T.size() == 1) lone_all.push_back(c.T[0]);
        }
        int lone_slot = 0, lone_reg = 0;
        for (int c : lone_all) (reg[c] >= 0 ? lone_reg : lone_slot)++;
        // balance registers against slots parent by parent
        {
            int cr = 0, cs = 0;
            for (size_t p = 0; p < ch.size(); ++p) {
                const Child& c = ch[p];
                if (c.lone) {
                    (reg[c.F[0]] >= 0 ? cr : cs)++;
                    continue;
                }
                int best = -1, bk = 1 << 30, br = 0, bs = 0;
                for (size_t o = 0; o < plans[p].size(); ++o) {
                    const int no = nout_of(c, plans[p][o].first), ni = nin_of(c, plans[p][o].second);
                    const int r1 = cr + (int)c.F.size() - no + ni, s1 = cs + (int)c.T.size() - ni + no;
                    if (std::abs(r1 - s1) < bk) {
                        bk = std::abs(r1 - s1);
                        best = (int)o;
                        br = r1;
                        bs = s1;
                    }
                }
                choice[p] = plans[p][best];
                cr = br;
                cs = bs;
            }
        }
        struct Tot {
            int r, s, nfs, nfg, nfs_raw;
        };
        auto totals = [&](const std::vector<std::pair<int, int>>& chs) {
            Tot t{0, 0, 0, 0, 0};
            int singles = 0, left = 0;
            for (size_t p = 0; p < ch.size(); ++p) {
                const Child& c = ch[p];
                if (c.lone) {
                    (reg[c.F[0]] >= 0 ? t.r : t.s)++;
                    continue;
                }
                const int no = nout_of(c, chs[p].first), ni = nin_of(c, chs[p].second);
                t.r += (int)c.F.size() - no + ni;
                t.s += (int)c.T.size() - ni + no;
                if (no == 1 && ni == 0) ++singles;
                left += std::max(0, ni - no);
            }
            const int m = std::min(singles, left);
            t.nfs = singles - m;
            t.nfg = left - m;
            t.nfs_raw = t.nfs;
            if (t.s > NS) {   // park lone LDS columns in free (or vacated) groups
                const int k = std::min({t.s - NS, lone_slot, (int)free_g.size() - t.nfg + t.nfs});
                if (k > 0) {
                    t.r += k;
                    t.s -= k;
                    t.nfg += k;
                }
            } else if (t.r > NG) {   // park lone register columns in free slots
                const int k = std::min({t.r - NG, lone_reg, (int)free_s.size() - t.nfs});
                if (k > 0) {
                    t.r -= k;
                    t.s += k;
                    t.nfs += k;
                }
            }
            return t;
        };
        auto over = [&](const Tot& t) {
            return std::max(0, t.r - NG) + std::max(0, t.s - NS) + std::max(0, t.nfs - (int)free_s.size()) +
                   std::max(0, t.nfg - (int)free_g.size() - t.nfs_raw);
        };
        for (int it = 0; it < 4 * (int)ch.size() + 4 && over(totals(choice)) > 0; ++it) {
            const int o0 = over(totals(choice));
            int bp = -1, bo = -1, bv = o0;
            for (size_t p = 0; p < ch.size(); ++p)
                for (size_t o = 0; o < plans[p].size(); ++o) {
                    if (plans[p][o] == choice[p]) continue;
                    auto trial = choice;
                    trial[p] = plans[p][o];
                    const int v = over(totals(trial));
                    if (v < bv) {
                        bv = v;
                        bp = (int)p;
                        bo = (int)o;
                    }
                }
            if (bp < 0) return false;
            choice[bp] = plans[bp][bo];
        }
        const Tot tt = totals(choice);
        if (over(tt) > 0) return false;
        // raw counts before parking decide how many lone columns are parked
        int r0 = 0, s0 = 0;
        for (size_t p = 0; p < ch.size(); ++p) {
            const Child& c = ch[p];
            if (c.lone) {
                (reg[c.F[0]] >= 0 ? r0 : s0)++;
                continue;
            }
            const int no = nout_of(c, choice[p].first), ni = nin_of(c, choice[p].second);
            r0 += (int)c.F.size() - no + ni;
            s0 += (int)c.T.size() - ni + no;
        }
        int park_s2r = std::max(0, s0 - NS), park_r2s = std::max(0, r0 - NG);
        // ---- apply: new holders and each group's action (write X / read Y)
        std::vector<int> nreg(n, -1), nslot(n, -1);
        std::vector<int> fg(free_g.begin(), free_g.end()), fs(free_s.begin(), free_s.end());
        size_t fgi = 0, fsi = 0;
        std::vector<int> singles, left_ins;
        uint32_t* tr = &S.trans[(size_t)(L + 1) * NG];
        auto act_write = [&](int g, int x) { tr[g] |= kTrWrite | (uint32_t)x; };
        auto act_read = [&](int g, int y) { tr[g] |= kTrRead | ((uint32_t)y << 8); };
        if (L + 1 >= kMaxLev) return false;
        std::vector<Seg> nsegs;
        for (size_t p = 0; p < ch.size(); ++p) {
            const Child& c = ch[p];
            if (c.lone) {
                nsegs.push_back(Seg{c.F, 1});
                continue;
            }
            const int fF = choice[p].first, fT = choice[p].second;
            const int no = nout_of(c, fF), ni = nin_of(c, fT);
            if (c.F.size() >= 2)
                for (int x = 0; x < (int)c.F.size() - no; ++x) nreg[c.F[x]] = reg[c.F[x]];
            if (c.T.size() >= 2)
                for (int x = ni; x < (int)c.T.size(); ++x) nslot[c.T[x]] = slot[c.T[x]];
            for (int x = 0; x < std::min(no, ni); ++x) {   // swap: out x into in x's slot
                const int o = c.F[c.F.size() - no + x], in = c.T[x];
                nreg[in] = reg[o];
                nslot[o] = slot[in];
                act_write(reg[o], slot[in]);
                act_read(reg[o], slot[in]);
            }
            for (int x = no; x < ni; ++x) left_ins.push_back(c.T[x]);
            if (no == 1 && ni == 0) singles.push_back(c.F[c.F.size() - 1]);
            nsegs.push_back(Seg{c.F, c.F.size() >= 2 ? fF : 1});
            nsegs.push_back(Seg{c.T, c.T.size() >= 2 ? fT : 1});
        }
        size_t si = 0, li = 0;
        for (; si < singles.size() && li < left_ins.size(); ++si, ++li) {   // cross-parent swaps
            const int o = singles[si], in = left_ins[li];
            nreg[in] = reg[o];
            nslot[o] = slot[in];
            act_write(reg[o], slot[in]);
            act_read(reg[o], slot[in]);
        }
        for (; li < left_ins.size(); ++li) {
            if (fgi >= fg.size()) return false;
            const int g = fg[fgi++];
            nreg[left_ins[li]] = g;
            act_read(g, slot[left_ins[li]]);
        }
        for (; si < singles.size(); ++si) {
            if (fsi >= fs.size()) return false;
            const int o = singles[si], x = fs[fsi++];
            nslot[o] = x;
            act_write(reg[o], x);
            fg.push_back(reg[o]);   // vacated: may read a parked lone column (write X, then read Y)
        }
        for (int c : lone_all) {
            if (reg[c] >= 0) {
                if (park_r2s > 0) {
                    if (fsi >= fs.size()) return false;
                    const int x = fs[fsi++];
                    nslot[c] = x;
                    act_write(reg[c], x);
                    --park_r2s;
                } else {
                    nreg[c] = reg[c];
                }
            } else {
                if (park_s2r > 0) {
                    if (fgi >= fg.size()) return false;
                    const int g = fg[fgi++];
                    nreg[c] = g;
                    act_read(g, slot[c]);
                    --park_s2r;
                } else {
                    nslot[c] = slot[c];
                }
            }
        }
        reg.swap(nreg);
        slot.swap(nslot);
        segs.swap(nsegs);
    }
    S.end_g.assign(NG, kNone);
    S.end_s.assign(NS, kNone);
    for (int c = 0; c < n; ++c) {
        if (reg[c] >= 0) S.end_g[reg[c]] = (uint32_t)c;
        if (slot[c] >= 0) S.end_s[slot[c]] = (uint32_t)c;
    }
    return true;
}

// Replays a schedule on column labels: the level-0 layout, every level's steps (each pair met
// once, no traveler used twice in a step, travelers read from their recorded slots) and every
// transition (a slot is written only if free at the level change or read by the same group; no
// slot read twice; the end layout as recorded).  Returns the steps per sweep, or -1.
int verify_schedule(const Schedule& S, int NG, int NS) {
    const int n = S.n;
    if (n < 2 || S.nlev < 1) return -1;
    std::vector<int> gcol(NG, -1), scol(NS, -1);
    for (int g = 0; g < S.f0; ++g) gcol[g] = g;
    for (int x = 0; x < n - S.f0; ++x) scol[x] = S.f0 + x;
    std::vector<uint8_t> met((size_t)n * n, 0);
    long pairs = 0;
    int steps = 0;
    for (int L = 0; L < S.nlev; ++L) {
        if (L > 0) {   // transition
            const uint32_t* tr = &S.trans[(size_t)L * NG];
            std::vector<int> ngcol = gcol, nscol = scol;
            std::vector<int> wr(NS, 0), rd(NS, 0);
            for (int g = 0; g < NG; ++g) {
                if (tr[g] & kTrRead) ++rd[(tr[g] >> 8) & 0xFF];
                if (tr[g] & kTrWrite) ++wr[tr[g] & 0xFF];
            }
            for (int x = 0; x < NS; ++x)
                if (wr[x] > 1 || rd[x] > 1) return -1;
            for (int g = 0; g < NG; ++g) {
                const bool w = tr[g] & kTrWrite, r = tr[g] & kTrRead;
                const int X = tr[g] & 0xFF, Y = (tr[g] >> 8) & 0xFF;
                if (w && (X >= NS || gcol[g] < 0)) return -1;
                if (w && scol[X] >= 0 && !(r && Y == X)) return -1;   // written slot busy, not a swap
                if (r && (Y >= NS || scol[Y] < 0)) return -1;
                if (r && !w && gcol[g] >= 0) return -1;              // reading group must be free or write first
                if (w && rd[X] && !(r && Y == X)) return -1;         // someone else reads it this phase
                if (r && wr[Y] && !(w && X == Y)) return -1;
            }
            for (int g = 0; g < NG; ++g) {
                const bool w = tr[g] & kTrWrite, r = tr[g] & kTrRead;
                const int X = tr[g] & 0xFF, Y = (tr[g] >> 8) & 0xFF;
                if (r) nscol[Y] = -1;
                if (w) ngcol[g] = -1;
            }
            for (int g = 0; g < NG; ++g) {
                const bool w = tr[g] & kTrWrite, r = tr[g] & kTrRead;
                const int X = tr[g] & 0xFF, Y = (tr[g] >> 8) & 0xFF;
                if (w) nscol[X] = gcol[g];
                if (r) ngcol[g] = scol[Y];
            }
            gcol.swap(ngcol);
            scol.swap(nscol);
        }
        const uint32_t* role = &S.role[(size_t)L * NG];
        int FL = 0;
        for (int g = 0; g < NG; ++g)
            if (role[g] & kRoleActive) FL = std::max(FL, (int)((role[g] >> 8) & 0xFF));
        if (FL != S.FL[L]) return -1;
        for (int j = 0; j < FL; ++j) {
            std::vector<uint8_t> used(NS, 0);
            for (int g = 0; g < NG; ++g) {
                if (!(role[g] & kRoleActive)) continue;
                const int i = role[g] & 0xFF, P = (role[g] >> 8) & 0xFF, t = (role[g] >> 16) & 0xFF,
                          base = (role[g] >> 24) & 0x7F;
                if (gcol[g] < 0 || i >= P) return -1;
                if (j >= P) continue;
                const int x = (i + j) % P;
                if (x >= t) continue;
                const int sl = base + x;
                if (sl >= NS || scol[sl] < 0 || used[sl]) return -1;
                used[sl] = 1;
                int a = gcol[g], b = scol[sl];
                if (a == b) return -1;
                if (a > b) std::swap(a, b);
                if (met[(size_t)a * n + b]) return -1;
                met[(size_t)a * n + b] = 1;
                ++pairs;
            }
        }
        steps += FL;
    }
    if (pairs != (long)n * (n - 1) / 2) return -1;
    for (int g = 0; g < NG; ++g)
        if ((gcol[g] < 0 ? kNone : (uint32_t)gcol[g]) != S.end_g[g]) return -1;
    for (int x = 0; x < NS; ++x)
        if ((scol[x] < 0 ? kNone : (uint32_t)scol[x]) != S.end_s[x]) return -1;
    return steps;
}

// The device table of one bucket: STRIDE words per k in [KLO, KHI]; nlev = kNone where the split
// layout does not take k.  Built once per process, copied to each context's device on first use.
template <int EMAX>
const std::vector<uint32_t>& host_table(int* kmax_ok) {
    using G = SplitGeom<EMAX>;
    static std::vector<uint32_t> tab;
    static int ok_hi = 0;
    static std::once_flag once;
    std::call_once(once, [] {
        tab.assign((size_t)(G::KHI - G::KLO + 1) * G::STRIDE, 0u);
        ok_hi = G::KLO - 1;
        bool contiguous = true;
        for (int k = G::KLO; k <= G::KHI; ++k) {
            uint32_t* t = &tab[(size_t)(k - G::KLO) * G::STRIDE];
            Schedule S;
            const bool built = build_schedule(k, G::NG, G::NS, S);
            const int steps = built ? verify_schedule(S, G::NG, G::NS) : -1;
            if (steps < 0) {
                t[0] = kNone;
                contiguous = false;
                continue;
            }
            if (contiguous) ok_hi = k;
            t[0] = (uint32_t)S.nlev;
            t[1] = (uint32_t)S.f0;
            for (int L = 0; L < kMaxLev; ++L) t[G::OFF_FL + L] = (uint32_t)S.FL[L];
            std::copy(S.role.begin(), S.role.end(), t + G::OFF_ROLE);
            std::copy(S.trans.begin(), S.trans.end(), t + G::OFF_TR);
            std::copy(S.end_g.begin(), S.end_g.end(), t + G::OFF_ENDG);
            std::copy(S.end_s.begin(), S.end_s.end(), t + G::OFF_ENDS);
        }
    });
    *kmax_ok = ok_hi;
    return tab;
}

// ------------------------------------------------------------------------------------------------
// Device
// FINISH: the refinement (cf_eigen.hip 4b) and the epilogue (5) run here too, from the slot through
// LDS row blocks, instead of in eigen_kernel's RESUME instantiation (one user per CU).
template <int EMAX, bool FINISH>
__global__ __launch_bounds__(SplitGeom<EMAX>::NT, SplitGeom<EMAX>::WPE) void split_sweep_kernel(EigenArgs a,
                                                                                             const uint32_t* sched) {
    using G = SplitGeom<EMAX>;
    constexpr int NR = G::NR, E2 = G::E2, NG = G::NG, NT = G::NT, NS = G::NS, LD = G::LD;
    constexpr int NW = NT / 64;
    extern __shared__ float smem[];
    float* Bs = smem;
    float* s_nrm = Bs + (size_t)NS * LD;   // traveling columns: tracked squared norm, drift (by slot)
    float* s_dev = s_nrm + NS;
    float* s_cn = s_dev + NS;              // fresh squared norm and drift by column label
    float* s_cd = s_cn + NR;
    float* s_s = s_cd + NR;
    float* s_l2d = s_s + NR;
    uint32_t* s_item = reinterpret_cast<uint32_t*>(s_l2d + NR);
    int* s_map = reinterpret_cast<int*>(s_item + NR);
    int* s_flag = s_map + NR;
    // phase stamps of thread 0 (cf_debug_stats) in LDS, off the VGPR budget
    unsigned long long* s_stamp = reinterpret_cast<unsigned long long*>(s_flag + 4);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int g = tid / kGroup;
    const int lig = tid % kGroup;
    if (a.stats && tid == 0) s_stamp[0] = __builtin_amdgcn_s_memtime();
    if (a.only_flag && !a.only_flag[blockIdx.x]) return;
    const uint32_t u = a.order[a.first + blockIdx.x];
    const uint64_t base = a.item_off[u];
    const int k = (int)(a.item_off[u + 1] - base);
    if (k < G::KLO || k > G::KHI) return;   // the launcher admits none (host-checked)
    const uint32_t* tab = sched + (size_t)(k - G::KLO) * G::STRIDE;
    const int nlev = (int)tab[0];
    const int f0 = (int)tab[1];
    float* hb = a.evecs + a.evec_off[u];    // k x k: W row-major, then B column-major

    // ---- 1. gather W (row i = w(item_i -> item_j)) into the slot, complement masks ----------
    for (int i = tid; i < k; i += NT) s_item[i] = a.items[base + i];
    if (tid == 0) {
        s_flag[0] = 0;
        s_flag[1] = 0;   // the largest sig written (float bits, all positive)
    }
    __syncthreads();
    const bool masks = a.cmask_out && 3 * (base + (uint64_t)k) <= a.cmask_words && u < a.cmask_users;
    if (masks && wave == 0) {
        const uint64_t fp = cf_items_fp(s_item, k, base, lane);
        if (lane == 0) a.cmask_fp[u] = fp;
    }
    // W rows go to the slot and, RB at a time, through LDS (the slot area, LDT = k | 1: a thread
    // per row reads its row conflict-free) for the degree and sig_min passes
    const int LDT = k | 1;
    const int RB = (NS * LD) / LDT;
    float* tile = Bs;
    for (int r0 = 0; r0 < k; r0 += RB) {
        const int rb = min(RB, k - r0);
        // four rows per wave at a time: all twelve graph loads in flight before the stores (the
        // compiler may not move a row's loads above the previous row's stores to the slot)
        for (int i0 = r0 + 4 * wave; i0 < r0 + rb; i0 += 4 * NW) {
            float w[4][3];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int i = i0 + q;
                const GraphRow row = a.graph.row(s_item[i < r0 + rb ? i : r0]);
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const int j = 64 * t + lane;
                    w[q][t] = (i < r0 + rb && j < k) ? row[s_item[j]] : 0.0f;
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int i = i0 + q;
                if (i >= r0 + rb) break;
                float* wr = hb + (size_t)i * k;
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const int j = 64 * t + lane;
                    if (j < k) {
                        wr[j] = w[q][t];
                        tile[(i - r0) * LDT + j] = w[q][t];
                    }
                    if (masks) {
                        // the predictor's mask words of row i (cf_eigen.hip stage 1)
                        const unsigned long long bal = __ballot(j < k && !((double)w[q][t] > 0.1));
                        if (lane == 0) a.cmask_out[3 * (base + i) + t] = bal;
                    }
                }
            }
        }
        __syncthreads();
        // ---- 2a. degrees (fp64, j in order), s, L2 diagonal: cf_eigen.hip stage 2
        for (int i = r0 + tid; i < r0 + rb; i += NT) {
            const float* wr = tile + (i - r0) * LDT;
            double d = 0.0;
            for (int j = 0; j < k; ++j) d += (double)wr[j];
            if (d == 0.0) d = 1.0;                       // (:137-140)
            const double s = sqrt(1.0 / d);              // (:149-153)
            s_s[i] = (float)s;
            s_l2d[i] = (float)((s * (d - (double)wr[i])) * s);
        }
        __syncthreads();
    }
    // ---- 2b. sig_min from the full rows (every s_j known): the rows again, from the slot
    for (int r0 = 0; r0 < k; r0 += RB) {
        const int rb = min(RB, k - r0);
        if (r0 > 0 || rb < k) {   // a single block is still in LDS
            for (int idx = tid; idx < rb * k; idx += NT) {
                const int i = idx / k, j = idx - i * k;
                tile[i * LDT + j] = hb[(size_t)(r0 + i) * k + j];
            }
            __syncthreads();
        }
        for (int i = r0 + tid; i < r0 + rb; i += NT) {
            const float* wr = tile + (i - r0) * LDT;
            const float si = s_s[i];
            float acc = 0.0f;
            for (int j = 0; j < k; ++j) {
                const float l2 = (j == i) ? s_l2d[i] : -(si * wr[j]) * s_s[j];
                acc = fmaf(l2, l2, acc);
            }
            const float sg = (float)((double)sqrtf(acc) + 0.01);   // (:172-176, :182)
            if (a.sigs) a.sigs[base + i] = sg;
            if (FINISH) atomicMax(&s_flag[1], __float_as_int(sg));
        }
        __syncthreads();
    }

    // ---- 3. B = sym_lower(L2) + I, 64 columns at a time: B(r, c) = -(s_max W(max, min)) s_min --
    // (cf_eigen.hip stage 3).  Tile column cc of the block holds B(:, c0 + cc); it is written over
    // rows c0.. of the row-major W, which no later block reads (they need W(r, c) with r >= their
    // c0, or their own rows).
    {
        for (int c0 = 0; c0 < k; c0 += G::CB) {
            const int cb = min(G::CB, k - c0);
            // r > c: W(r, c), lanes over the block's columns (a row segment per pass)
            for (int idx = tid; idx < (k - c0) * G::CB; idx += NT) {
                const int r = c0 + idx / G::CB, cc = idx % G::CB, c = c0 + cc;
                if (cc < cb && c < r) tile[cc * LDT + r] = -(s_s[r] * hb[(size_t)r * k + c]) * s_s[c];
            }
            // r < c: W(c, r), a wave per column, lanes down its row of W; the diagonal
            for (int cc = wave; cc < cb; cc += NW) {
                const int c = c0 + cc;
                const float* wr = hb + (size_t)c * k;
                for (int r = lane; r < c; r += 64) tile[cc * LDT + r] = -(s_s[c] * wr[r]) * s_s[r];
                if (lane == 0) tile[cc * LDT + c] = s_l2d[c] + 1.0f;
            }
            __syncthreads();
            for (int cc = wave; cc < cb; cc += NW) {
                float* out = hb + (size_t)(c0 + cc) * k;
                for (int r = lane; r < k; r += 64) out[r] = tile[cc * LDT + r];
            }
            // squared norms in the sweeps' float2 layout (rows 16e + 2lig, +1)
            for (int cc = g; cc < cb; cc += NG) {
                f2 acc = {0.f, 0.f};
#pragma unroll
                for (int e = 0; e < E2; ++e) {
                    const int r = 16 * e + 2 * lig;
                    const f2 x = {r < k ? tile[cc * LDT + r] : 0.0f, r + 1 < k ? tile[cc * LDT + r + 1] : 0.0f};
                    acc = __builtin_elementwise_fma(x, x, acc);
                }
                const float nc = pair_sum(acc.x + acc.y);
                if (lig == 0) {
                    s_cn[c0 + cc] = nc;
                    s_cd[c0 + cc] = 0.0f;
                }
            }
            __syncthreads();
        }
    }
    if (a.stats && tid == 0) s_stamp[1] = __builtin_amdgcn_s_memtime();

    // ---- 4. sweeps ----------------------------------------------------------------------------
    // uniform: kept in scalar registers (readfirstlane), off the VGPR budget of the sweeps
    auto uni = [](float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); };
    const float tol = a.tol_scale * sqrtf((float)k) * 2.384185791015625e-07f;   // sqrt(k) * 2^-22
    const float tol2 = uni(tol * tol);
    const bool refine = a.refine && k > 1;
    const float stop2 = uni(refine ? a.stop_rel * a.stop_rel : kSigRot2 * tol * tol);
    const float close2 = uni(refine ? a.close_sigrot * a.close_sigrot * tol * tol : stop2);
    const float dclose2 = uni(refine ? 2.0f * a.refine_delta * a.refine_delta : -1.0f);
    // column c of B in the slot, rows 16e + 2lig, +1 of this lane (zero past k)
    auto load_col = [&](int c, f2* x) {
        const float* src = hb + (size_t)c * k;
#pragma unroll
        for (int e = 0; e < E2; ++e) {
            const int r = 16 * e + 2 * lig;
            x[e] = f2{r < k ? src[r] : 0.0f, r + 1 < k ? src[r + 1] : 0.0f};
        }
    };
    int sweep = 0;
    int steps_sweep = 0;
    for (int L = 0; L < nlev; ++L) steps_sweep += (int)tab[G::OFF_FL + L];
    for (; sweep < a.max_sweeps; ++sweep) {
        // norm order (cf_eigen.hip's sorted sweeps): s_map[rank] = column
        if (a.sort_sweeps) {
            const bool asc = a.sort_sweeps == 2;
            constexpr int RB = (NR + 63) / 64;
            float ni[RB];
#pragma unroll
            for (int r = 0; r < RB; ++r) ni[r] = (64 * r + lane < k) ? s_cn[64 * r + lane] : -1.0f;
            for (int j = wave; j < k; j += NW) {
                const float nj = s_cn[j];
                int rank = 0;
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const int i = 64 * r + lane;
                    const bool before = asc ? ni[r] < nj : ni[r] > nj;
                    rank += __popcll(__ballot(i < k && (before || (ni[r] == nj && i < j))));
                }
                if (lane == 0) s_map[rank] = j;
            }
        } else {
            for (int j = tid; j < k; j += NT) s_map[j] = j;
        }
        __syncthreads();
        // level 0: traveling rank f0 + x in slot x, then fixed F[g] = rank g in registers
        if (g < k - f0) {
            const int c = s_map[f0 + g];
            const float* src = hb + (size_t)c * k;
            f2* dst = reinterpret_cast<f2*>(Bs + (size_t)g * LD);
#pragma unroll
            for (int e = 0; e < E2; ++e) {
                const int r = 16 * e + 2 * lig;
                lds_st(dst + kGroup * e + lig, f2{r < k ? src[r] : 0.0f, r + 1 < k ? src[r + 1] : 0.0f});
            }
            if (lig == 0) {
                s_nrm[g] = s_cn[c];
                s_dev[g] = s_cd[c];
            }
        }
        f2 xp[E2];
        float devp = 0.0f, al = 0.0f;
        if (g < f0) {
            const int c = s_map[g];
            load_col(c, xp);
            devp = s_cd[c];
        } else {
#pragma unroll
            for (int e = 0; e < E2; ++e) xp[e] = f2{0.f, 0.f};
        }
        __syncthreads();
        for (int L = 0; L < nlev; ++L) {
            if (L > 0) {
                // level change: write this group's column to slot X and/or read slot Y (a swap
                // when X == Y: every lane reads its rows before it writes them)
                const uint32_t tr = tab[G::OFF_TR + L * NG + g];
                if (tr & (kTrRead | kTrWrite)) {
                    const bool rd = tr & kTrRead, wr = tr & kTrWrite;
                    const f2* src = reinterpret_cast<const f2*>(Bs + (size_t)((tr >> 8) & 0xFF) * LD);
                    f2* dst = reinterpret_cast<f2*>(Bs + (size_t)(tr & 0xFF) * LD);
                    const float dy = rd ? s_dev[(tr >> 8) & 0xFF] : 0.0f;
                    const float ny = rd ? s_nrm[(tr >> 8) & 0xFF] : 0.0f;
                    // element by element: a lane reads its rows of Y before it writes the same rows
                    // of X, and no other group touches X or Y in this phase
#pragma unroll
                    for (int e = 0; e < E2; ++e) {
                        const f2 y = rd ? lds_ld(src + kGroup * e + lig) : f2{0.f, 0.f};
                        if (wr) lds_st(dst + kGroup * e + lig, xp[e]);
                        if (rd) xp[e] = y;
                    }
                    if (wr && lig == 0) {
                        s_dev[tr & 0xFF] = devp;
                        s_nrm[tr & 0xFF] = al;
                    }
                    if (rd) {
                        devp = dy;
                        al = ny;
                    }
                }
                __syncthreads();
            }
            const uint32_t role = tab[G::OFF_ROLE + L * NG + g];
            const int FL = (int)tab[G::OFF_FL + L];
            const bool active = role & kRoleActive;
            const int fi = role & 0xFF, P = (role >> 8) & 0xFF, t = (role >> 16) & 0xFF, bsl = (role >> 24) & 0x7F;
            if (active) {   // fresh norm of the fixed column at every level start
                f2 al2 = {0.f, 0.f};
#pragma unroll
                for (int e = 0; e < E2; ++e) al2 = __builtin_elementwise_fma(xp[e], xp[e], al2);
                al = pair_sum(al2.x + al2.y);
            }
            // inactive groups have P = t = 0: no step of theirs is live
            int ti = fi;
            for (int step = 0; step < FL; ++step) {
                if (step < P && ti < t) {
                    const int q = bsl + ti;
                    f2* bq = reinterpret_cast<f2*>(Bs + (size_t)q * LD) + lig;
                    const float dq = s_dev[q];
                    const float be = s_nrm[q];
                    f2 xq[E2];
                    f2 ga2[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
                    for (int e = 0; e < E2; ++e) xq[e] = lds_ld(bq + kGroup * e);
#pragma unroll
                    for (int e = 0; e < E2; ++e) ga2[e & 1] = __builtin_elementwise_fma(xp[e], xq[e], ga2[e & 1]);
                    const f2 gs = ga2[0] + ga2[1];
                    const float ga = pair_sum(gs.x + gs.y);
                    if (ga * ga > tol2 * (al * be)) {
                        // cf_eigen.hip stage 4: t = 2 ga sign(be - al) / (|be - al| + sqrt((be - al)^2 + 4 ga^2)),
                        // hardware rcp / rsq / sqrt, the scale drift c^2 + s^2 - 1 tracked per column
                        const float dd = be - al;
                        const float r = __builtin_amdgcn_sqrtf(fmaf(dd, dd, 4.0f * ga * ga));
                        const float tt = (dd < 0.0f ? -2.0f * ga : 2.0f * ga) * __builtin_amdgcn_rcpf(fabsf(dd) + r);
                        const float c = __builtin_amdgcn_rsqf(fmaf(tt, tt, 1.0f));
                        const float sn = c * tt;
                        const f2 c2 = {c, c}, s2 = {sn, sn}, ns2 = {-sn, -sn};
#pragma unroll
                        for (int e = 0; e < E2; ++e) {
                            const f2 np = __builtin_elementwise_fma(ns2, xq[e], c2 * xp[e]);
                            lds_st(bq + kGroup * e, __builtin_elementwise_fma(s2, xp[e], c2 * xq[e]));
                            xp[e] = np;
                        }
                        const float delta = fmaf(sn, sn, fmaf(c, c, -1.0f));
                        const float cc = c * c, ss = sn * sn;
                        const float ndp = delta + fmaf(cc, devp, ss * dq);
                        const float csg = 2.0f * c * sn * ga;
                        const float nal = fmaf(cc, al, fmaf(ss, be, -csg));
                        if (lig == 0) {
                            s_dev[q] = delta + fmaf(ss, devp, cc * dq);
                            s_nrm[q] = fmaf(ss, al, fmaf(cc, be, csg));
                            const float g2 = ga * ga, ab = al * be, dab = be - al;
                            if (g2 > stop2 * ab || (g2 > close2 * ab && dab * dab <= dclose2 * (al + be))) s_flag[0] = 1;
                        }
                        devp = ndp;
                        al = nal;
                    }
                }
                __syncthreads();
                if (++ti == P) ti = 0;
            }
        }
        // sweep end: every column back to the slot at its label, with its fresh norm and drift
        const uint32_t end_g = tab[G::OFF_ENDG + g];
        const uint32_t end_s = g < NS ? tab[G::OFF_ENDS + g] : kNone;
        if (end_g != kNone) {
            float* dst = hb + (size_t)end_g * k;
            f2 acc = {0.f, 0.f};
#pragma unroll
            for (int e = 0; e < E2; ++e) {
                const int r = 16 * e + 2 * lig;
                if (r < k) dst[r] = xp[e].x;
                if (r + 1 < k) dst[r + 1] = xp[e].y;
                acc = __builtin_elementwise_fma(xp[e], xp[e], acc);
            }
            const float nc = pair_sum(acc.x + acc.y);
            if (lig == 0) {
                s_cn[end_g] = nc;
                s_cd[end_g] = devp;
            }
        }
        if (end_s != kNone) {
            const f2* src = reinterpret_cast<const f2*>(Bs + (size_t)g * LD);
            float* dst = hb + (size_t)end_s * k;
            f2 acc = {0.f, 0.f};
#pragma unroll
            for (int e = 0; e < E2; ++e) {
                const f2 x = lds_ld(src + kGroup * e + lig);
                const int r = 16 * e + 2 * lig;
                if (r < k) dst[r] = x.x;
                if (r + 1 < k) dst[r + 1] = x.y;
                acc = __builtin_elementwise_fma(x, x, acc);
            }
            const float nc = pair_sum(acc.x + acc.y);
            if (lig == 0) {
                s_cn[end_s] = nc;
                s_cd[end_s] = s_dev[g];
            }
        }
        __syncthreads();
        const int rotated = s_flag[0];
        __syncthreads();
        if (!rotated) break;
        if (tid == 0) s_flag[0] = 0;
        __syncthreads();
    }
    if (a.stats && tid == 0) s_stamp[2] = __builtin_amdgcn_s_memtime();
    if constexpr (!FINISH) {
        // ---- 5. drifts for the refinement / epilogue kernel (eigen_kernel<.., RESUME>)
        for (int j = tid; j < k; j += NT) a.evals[base + j] = s_cd[j];
    } else {
        // ---- 5'. first-order Gram refinement (cf_eigen.hip 4b) from the column-major slot ------
        float* s_mu = s_l2d;   // free after the assembly
        float* tile = Bs;      // the slot area, free after the last sweep
        const int nb = (k + 15) >> 4;
        const int m16 = lane & 15, kq = lane >> 4;
        const int jc = wave * 16 + m16;   // this lane's column (wave < nb; NW >= nb)
        const bool jv = wave < nb && jc < k;
        f4 kv[EMAX];
#pragma unroll
        for (int I = 0; I < EMAX; ++I) kv[I] = f4{0.f, 0.f, 0.f, 0.f};
        if (refine) {
            for (int c = tid; c < k; c += NT) s_mu[c] = s_cn[c] / (1.0f + s_cd[c]);   // fresh mu^2
            // F = B^T B over row blocks of RB1 rows: column segments staged in LDS, the same 16-row
            // chunks in the same order as cf_eigen.hip's F loop
            constexpr int RB1 = (((NS * LD) / G::KHI - 4) / 16) * 16;
            constexpr int LDR1 = RB1 + 4;   // f4-aligned column segments
            static_assert(RB1 >= 16, "refinement row block");
            for (int R0 = 0; R0 < k; R0 += RB1) {
                __syncthreads();
                for (int idx = tid; idx < k * RB1; idx += NT) {
                    const int c = idx / RB1, r = idx - c * RB1;
                    tile[c * LDR1 + r] = (R0 + r < k) ? hb[(size_t)c * k + R0 + r] : 0.0f;
                }
                __syncthreads();
                if (wave < nb) {
                    const int nc16 = (min(RB1, k - R0) + 15) >> 4;
                    const f4* pj = reinterpret_cast<const f4*>(tile + (jv ? jc : 0) * LDR1 + 4 * kq);
                    for (int c = 0; c < nc16; ++c) {
                        const f4 y = jv ? pj[4 * c] : f4{0.f, 0.f, 0.f, 0.f};
                        // two row tiles per operand step (cf_eigen.hip takes four: the accumulators of
                        // all EMAX tiles already hold 4 * EMAX of this kernel's 80 registers)
#pragma unroll
                        for (int I0 = 0; I0 < EMAX; I0 += 2) {
                            f4 x[2];
#pragma unroll
                            for (int g2 = 0; g2 < 2; ++g2) {
                                const int ci = (I0 + g2) * 16 + m16;
                                x[g2] = (I0 + g2 < nb && ci < k) ? reinterpret_cast<const f4*>(tile + ci * LDR1 + 4 * kq)[4 * c]
                                                                 : f4{0.f, 0.f, 0.f, 0.f};
                            }
#pragma unroll
                            for (int t = 0; t < 4; ++t)
#pragma unroll
                                for (int g2 = 0; g2 < 2; ++g2)
                                    if (I0 + g2 < EMAX && I0 + g2 < nb)
                                        kv[I0 + g2] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[g2][t], y[t], kv[I0 + g2], 0, 0, 0);
                        }
                    }
                }
            }
            // K(i, j) = F(i, j) / (mu_i^2 - mu_j^2), |mu_i - mu_j| > delta, i != j (cf_eigen.hip 4b)
            if (wave < nb) {
                const float muj2 = jv ? s_mu[jc] : 1.0f;
                const float muj = sqrtf(muj2);
                const float dlt = a.refine_delta;
                float ksq = 0.0f;
#pragma unroll
                for (int I = 0; I < EMAX; ++I)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = I * 16 + 4 * kq + r;
                        float kvv = 0.0f;
                        if (I < nb && jv && i < k && i != jc) {
                            const float mui2 = s_mu[i];
                            if (fabsf(sqrtf(mui2) - muj) > dlt) kvv = kv[I][r] / (mui2 - muj2);
                        }
                        kv[I][r] = -kvv;
                        ksq = fmaf(kvv, kvv, ksq);
                    }
                ksq += __shfl_xor(ksq, 16);
                ksq += __shfl_xor(ksq, 32);
                if (kq == 0 && jv) s_cd[jc] += ksq;
            }
        }
        __syncthreads();
        // the slot column-major -> row-major in place (pair swaps): the update and the output read
        // and write whole rows, which a row block owns
        for (int i = wave; i < k; i += NW)
            for (int jj = i + 1 + lane; jj < k; jj += 64) {
                const float x = hb[(size_t)i * k + jj], y = hb[(size_t)jj * k + i];
                hb[(size_t)i * k + jj] = y;
                hb[(size_t)jj * k + i] = x;
            }
        __syncthreads();
        if (refine) {
            // B(R, J) - B(R, :) K(:, J) for row blocks R of 48 rows, written back over rows R
            constexpr int RB3x = (((NS * LD) / G::KHI - 1) / 16) * 16;   // rows whose k columns fit the area
            constexpr int RB3 = RB3x < 48 ? RB3x : 48, LDR3 = RB3 + 1;
            static_assert(RB3 >= 16 && G::KHI * LDR3 <= NS * LD, "update row block");
            for (int R0 = 0; R0 < k; R0 += RB3) {
                for (int idx = tid; idx < RB3 * k; idx += NT) {
                    const int r = idx / k, c = idx - r * k;
                    tile[c * LDR3 + r] = (R0 + r < k) ? hb[(size_t)(R0 + r) * k + c] : 0.0f;
                }
                __syncthreads();
                if (wave < nb) {
                    f4 out[RB3 / 16];
#pragma unroll
                    for (int q = 0; q < RB3 / 16; ++q)
#pragma unroll
                        for (int r = 0; r < 4; ++r) out[q][r] = jv ? tile[jc * LDR3 + 16 * q + 4 * kq + r] : 0.0f;
#pragma unroll
                    for (int I = 0; I < EMAX; ++I) {
                        if (I < nb) {
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                const int c = I * 16 + 4 * kq + t;
#pragma unroll
                                for (int q = 0; q < RB3 / 16; ++q) {
                                    const float av = c < k ? tile[c * LDR3 + 16 * q + m16] : 0.0f;
                                    out[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, kv[I][t], out[q], 0, 0, 0);
                                }
                            }
                        }
                    }
                    if (jv)
#pragma unroll
                        for (int q = 0; q < RB3 / 16; ++q)
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int row = R0 + 16 * q + 4 * kq + r;
                                if (row < k) hb[(size_t)row * k + jc] = out[q][r];
                            }
                }
                __syncthreads();
            }
        }
        // ---- 6'. epilogue (cf_eigen.hip 5): fp64 norms and sign sums, rank, lim, the k x m block --
        for (int jj = tid; jj < k; jj += NT) {
            double acc = 0.0, sum = 0.0;
            for (int r = 0; r < k; ++r) {
                const double v = (double)hb[(size_t)r * k + jj];
                acc = fma(v, v, acc);
                sum += v;
            }
            const double nrm = sqrt(acc);
            s_mu[jj] = (float)(nrm / sqrt(1.0 + (double)s_cd[jj]));   // lambda_j + 1
            s_s[jj] = (float)((sum < 0.0 ? -1.0 : 1.0) / nrm);        // unit-normalises v_j, sum >= 0
        }
        __syncthreads();
        for (int jj = tid; jj < k; jj += NT) {
            const float mj = s_mu[jj];
            int rank = 0;
            for (int i = 0; i < k; ++i) {
                const float mi = s_mu[i];
                rank += (mi < mj) || (mi == mj && i < jj);
            }
            s_map[rank] = jj;
        }
        // lim = #{!(lambda > smm)} (cf_eigen.hip 5); smm = the largest sig written (sig + 0.01 rounded)
        const float smm = __int_as_float(s_flag[1]);
        const bool below = tid < k && !((double)(s_mu[tid] - 1.0f) > (double)smm);
        int lim = __syncthreads_count(below);
        if (lim < 2) lim = 2;
        if (tid == 0) a.m_out[u] = lim;
        const int m = min(lim, k);
        for (int r = tid; r < k; r += NT) a.evals[base + r] = r < m ? s_mu[s_map[r]] - 1.0f : 0.0f;
        // the k x m row-major block over the row-major Bref, rows in increasing order through LDS: a
        // block's output rows land on rows it or an earlier block held (m <= k)
        const int LDO = k + 1;
        const int RBo = (NS * LD) / LDO;
        for (int i0 = 0; i0 < k; i0 += RBo) {
            const int rb = min(RBo, k - i0);
            for (int idx = tid; idx < rb * k; idx += NT) {
                const int r = idx / k, c = idx - r * k;
                tile[r * LDO + c] = hb[(size_t)(i0 + r) * k + c];
            }
            __syncthreads();
            for (int idx = tid; idx < rb * lim; idx += NT) {
                const int r = idx / lim, cc = idx - r * lim;
                float v = 0.0f;
                if (cc < k) {
                    const int jj = s_map[cc];
                    v = tile[r * LDO + jj] * s_s[jj];
                }
                hb[(size_t)(i0 + r) * lim + cc] = v;
            }
            __syncthreads();
        }
    }
    if (a.stats && tid == 0) {
        const unsigned long long t3 = __builtin_amdgcn_s_memtime();
        atomicAdd(&a.stats[0], (unsigned long long)(sweep + 1));
        atomicAdd(&a.stats[1], 1ull);
        atomicMax(&a.stats[2], (unsigned long long)(sweep + 1));
        if (sweep >= a.max_sweeps) atomicAdd(&a.stats[3], 1ull);
        atomicAdd(&a.stats[4], s_stamp[1] - s_stamp[0]);
        atomicAdd(&a.stats[5], s_stamp[2] - s_stamp[1]);
        if (FINISH) atomicAdd(&a.stats[6], t3 - s_stamp[2]);
        atomicAdd(&a.stats[7], (unsigned long long)((sweep + 1) * steps_sweep));
    }
}

template <int EMAX, bool FINISH>
int launch_split_kernel(cf_ctx* ctx, const EigenArgs& a, uint32_t count, hipStream_t stream) {
    using G = SplitGeom<EMAX>;
    static bool configured = false;
    if (!configured) {
        CF_HIP_CHECK(ctx, hipFuncSetAttribute((const void*)split_sweep_kernel<EMAX, FINISH>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::bytes()));
        configured = true;
    }
    hipLaunchKernelGGL((split_sweep_kernel<EMAX, FINISH>), dim3(count), dim3(G::NT), G::bytes(), stream, a,
                       (const uint32_t*)ctx->d_split_sched[EMAX]);
    CF_HIP_CHECK(ctx, hipGetLastError());
    return CF_OK;
}

template <int EMAX>
int launch_emax_split(cf_ctx* ctx, const EigenArgs& a, uint32_t count, uint32_t kmax, hipStream_t stream,
                      bool* handled, bool* finished) {
    int ok_hi = 0;
    const std::vector<uint32_t>& tab = host_table<EMAX>(&ok_hi);
    if ((int)kmax > ok_hi) return CF_OK;   // not every k of the launch has a schedule
    if (!ctx->d_split_sched[EMAX]) {
        void* p = nullptr;
        CF_TRY(cf_malloc_evict(ctx, &p, tab.size() * sizeof(uint32_t), "split sweep schedule"));
        ctx->d_split_sched[EMAX] = static_cast<uint32_t*>(p);
        CF_HIP_CHECK(ctx, hipMemcpy(p, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    if (ctx->split_finish < 0) {   // CF_EIGEN_SPLIT_FINISH: 1 every bucket, 0 none, unset buckets <= 8
        const char* e = getenv("CF_EIGEN_SPLIT_FINISH");
        ctx->split_finish = !e ? 2 : (e[0] == '1') ? 1 : 0;
    }
    // buckets <= 8: their RESUME twin spills (eigen_kernel<8, .., true>: 320 VGPRs), and K's 4 * EMAX
    // accumulators fit beside the sweeps' registers; above, kernel B is faster
    if (ctx->split_finish == 1 || (ctx->split_finish == 2 && EMAX <= 8)) {
        CF_TRY((launch_split_kernel<EMAX, true>(ctx, a, count, stream)));
        *finished = true;
    } else {
        CF_TRY((launch_split_kernel<EMAX, false>(ctx, a, count, stream)));
    }
    *handled = true;
    return CF_OK;
}

}  // namespace

int launch_split_sweeps(cf_ctx* ctx, const EigenArgs& a, int emax, uint32_t count, uint32_t kmax, hipStream_t stream,
                        bool* handled, bool* finished) {
    *handled = false;
    *finished = false;
    if (a.mode != kUser || emax < kSplitEmaxLow || emax > 12 || count == 0) return CF_OK;
    if (ctx->eigen_split < 0) {   // CF_EIGEN_SPLIT: 0 off, else the smallest bucket (default kSplitEmaxMin)
        const char* e = getenv("CF_EIGEN_SPLIT");
        ctx->eigen_split = e ? atoi(e) : 1;
    }
    const int emin = ctx->eigen_split == 1 ? kSplitEmaxMin : ctx->eigen_split;
    if (!ctx->eigen_split || emax < emin) return CF_OK;
    switch (emax) {
        case 5: return launch_emax_split<5>(ctx, a, count, kmax, stream, handled, finished);
        case 6: return launch_emax_split<6>(ctx, a, count, kmax, stream, handled, finished);
        case 7: return launch_emax_split<7>(ctx, a, count, kmax, stream, handled, finished);
        case 8: return launch_emax_split<8>(ctx, a, count, kmax, stream, handled, finished);
        case 9: return launch_emax_split<9>(ctx, a, count, kmax, stream, handled, finished);
        case 10: return launch_emax_split<10>(ctx, a, count, kmax, stream, handled, finished);
        case 11: return launch_emax_split<11>(ctx, a, count, kmax, stream, handled, finished);
        case 12: return launch_emax_split<12>(ctx, a, count, kmax, stream, handled, finished);
        default: return CF_OK;
    }
}

}  // namespace cf_eig

using namespace cf_eig;

extern "C" int cf_set_eigen_split(cf_ctx* ctx, int enable) {
    if (!ctx) return CF_EINVAL;
    if (enable < 0 || (enable > 1 && (enable < kSplitEmaxLow || enable > 12))) return CF_EINVAL;
    ctx->eigen_split = enable;
    return CF_OK;
}

namespace {
template <int EMAX>
void geom_of(int* ng, int* ns, int* klo, int* khi) {
    *ng = SplitGeom<EMAX>::NG;
    *ns = SplitGeom<EMAX>::NS;
    *klo = SplitGeom<EMAX>::KLO;
    *khi = SplitGeom<EMAX>::KHI;
}
}  // namespace

extern "C" int cf_debug_split_schedule(int emax, int k, int* steps, int* levels, int* max_groups, int* max_slots) {
    int NG, NS, klo, khi;
    switch (emax) {
        case 5: geom_of<5>(&NG, &NS, &klo, &khi); break;
        case 6: geom_of<6>(&NG, &NS, &klo, &khi); break;
        case 7: geom_of<7>(&NG, &NS, &klo, &khi); break;
        case 8: geom_of<8>(&NG, &NS, &klo, &khi); break;
        case 9: geom_of<9>(&NG, &NS, &klo, &khi); break;
        case 10: geom_of<10>(&NG, &NS, &klo, &khi); break;
        case 11: geom_of<11>(&NG, &NS, &klo, &khi); break;
        case 12: geom_of<12>(&NG, &NS, &klo, &khi); break;
        default: return CF_ERANGE;
    }
    if (k < klo || k > khi) return CF_ERANGE;
    Schedule S;
    if (!build_schedule(k, NG, NS, S)) return CF_ERANGE;
    const int st = verify_schedule(S, NG, NS);
    if (st < 0) return CF_ERANGE;
    if (steps) *steps = st;
    if (levels) *levels = S.nlev;
    if (max_groups) *max_groups = S.max_groups;
    if (max_slots) *max_slots = S.max_slots;
    return CF_OK;
}
