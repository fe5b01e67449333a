// relabel.cpp — bank-aware relabelling of bit ids for the V2 kernels' LDS
// totals (host only).
//
// The V2 check-node scan reads total[col] with one ds_read_b64 per slot, every
// lane of the wave at once (decoder_v2.hip).  gfx950 services a 64-bit LDS
// read in two 32-lane halves, and within a half a double at index c occupies
// banks 2c, 2c + 1 (mod 64): lanes whose columns agree mod 32 but differ
// serialise (MI355X_MICROARCH.md §LDS).  With the reference's random codes
// the 32 columns of a half fall into 32 classes at random — about 3.5
// distinct addresses on the busiest bank per half.  The min-sum bit gather's
// message pass also ORs two bits per edge into the bit's code word
// (ds_or_b32 at byte c & ~3: bank (c >> 2) mod 32).
//
// Bit ids are free labels: the decode never depends on their order (a row's
// product runs in the row's CSR order and a bit's sum in ascending check
// order, src/qkd_ldpc_algorithm.cpp:57-62,78, whatever the labels), so the
// planner may renumber the columns so that every (wave, slot, half) group of
// the slot layout reads distinct banks.  Each column gets a residue class r
// (mod NR = 128): the read bank is r mod 32, the code-word bank (r >> 2) mod
// 32.  Starting from a balanced random assignment, a deterministic local
// search swaps the classes of two columns when that does not raise the summed
// cost (over groups and banks, (count - 1)^2 for count > 1: a 3-way conflict
// costs more than two 2-way ones, so the search drives every group's busiest
// bank down to 2).  A conflict-free layout (every class exactly once per
// group) is an exact-cover problem the random codes do not admit: on C2 the
// busiest-bank count per half goes from 3.5 (any fixed labelling of a random
// code) to 2.0.  Labels are then dealt class by class: class r gets r,
// r + NR, r + 2 NR, ...
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <random>
#include <vector>

#include "relabel.hpp"

namespace qldpc {

namespace {

constexpr int NR = 128;  // residue classes (4 x the 32 read banks: room for the code-word bank)
inline int bank_read(int r) { return r & 31; }
inline int bank_word(int r) { return (r >> 2) & 31; }

}  // namespace

std::vector<int32_t> bank_relabel(int n, const std::vector<RelabelGroup> &groups, uint64_t seed, long long iters,
                                  RelabelStats *stats) {
    std::vector<int32_t> lab(n);
    for (int i = 0; i < n; ++i) lab[i] = i;
    if (n < NR || groups.empty()) return lab;
    const int G = (int)groups.size();
    // incidences per column: (group, functions mask)
    std::vector<std::vector<std::pair<int, uint8_t>>> inc(n);
    for (int g = 0; g < G; ++g)
        for (const auto &mb : groups[g].members)
            if (mb.col >= 0 && mb.col < n) inc[mb.col].push_back({g, mb.fmask});
    // counts: [g][bank] for the read banks (f1) and the code-word banks (f2)
    std::vector<uint16_t> c1((size_t)G * 32, 0), c2((size_t)G * 32, 0);
    std::vector<int> res(n);
    // balanced initial classes: label i's class, shuffled over the columns
    std::mt19937_64 rng(seed);
    {
        std::vector<int> cls(n);
        for (int i = 0; i < n; ++i) cls[i] = i % NR;
        std::shuffle(cls.begin(), cls.end(), rng);
        res = cls;
    }
    auto exc = [](int c) { return c > 1 ? (c - 1) * (c - 1) : 0; };
    for (int g = 0; g < G; ++g)
        for (const auto &mb : groups[g].members) {
            const int r = mb.col >= 0 ? res[mb.col] : mb.fixed_res;
            if (mb.fmask & 1) ++c1[(size_t)g * 32 + bank_read(r)];
            if (mb.fmask & 2) ++c2[(size_t)g * 32 + bank_word(r)];
        }
    auto total_cost = [&]() {
        long long s = 0;
        for (size_t i = 0; i < c1.size(); ++i) s += exc(c1[i]) + exc(c2[i]);
        return s;
    };
    auto total_cycles = [&]() {
        long long s = 0;
        for (int g = 0; g < G; ++g) {
            int m1 = 0, m2 = 0;
            for (int b = 0; b < 32; ++b) {
                m1 = std::max<int>(m1, c1[(size_t)g * 32 + b]);
                m2 = std::max<int>(m2, c2[(size_t)g * 32 + b]);
            }
            s += m1 + m2;
        }
        return s;
    };
    const long long cost0 = total_cost(), cyc0 = total_cycles();
    // columns of each class, with positions (O(1) swaps)
    std::vector<std::vector<int>> of(NR);
    std::vector<int> pos(n);
    for (int i = 0; i < n; ++i) {
        pos[i] = (int)of[res[i]].size();
        of[res[i]].push_back(i);
    }
    // move column a to class r: returns the change in cost
    auto move = [&](int a, int r) -> int {
        const int r0 = res[a];
        int d = 0;
        for (const auto &gi : inc[a]) {
            const size_t base = (size_t)gi.first * 32;
            if (gi.second & 1) {
                uint16_t &o = c1[base + bank_read(r0)];
                d -= exc(o);
                --o;
                d += exc(o);
                uint16_t &q = c1[base + bank_read(r)];
                d -= exc(q);
                ++q;
                d += exc(q);
            }
            if (gi.second & 2) {
                uint16_t &o = c2[base + bank_word(r0)];
                d -= exc(o);
                --o;
                d += exc(o);
                uint16_t &q = c2[base + bank_word(r)];
                d -= exc(q);
                ++q;
                d += exc(q);
            }
        }
        res[a] = r;
        return d;
    };
    auto swap_pos = [&](int a, int b) {  // a, b exchanged their classes: fix the class lists
        const int ra = res[a], rb = res[b];
        std::swap(pos[a], pos[b]);
        of[ra][pos[a]] = a;
        of[rb][pos[b]] = b;
    };
    long long cost = cost0;
    std::uniform_int_distribution<int> pick_col(0, n - 1);
    std::uniform_real_distribution<double> u01(0.0, 1.0);
    long long it = 0, accepted = 0;
    for (; it < iters && cost > 0; ++it) {
        const int a = pick_col(rng);
        // a conflicting incidence of a (its read bank or code-word bank shared)
        int g = -1;
        for (const auto &gi : inc[a]) {
            const size_t base = (size_t)gi.first * 32;
            if (((gi.second & 1) && c1[base + bank_read(res[a])] > 1) ||
                ((gi.second & 2) && c2[base + bank_word(res[a])] > 1)) {
                g = gi.first;
                break;
            }
        }
        if (g < 0) continue;
        // a target class whose banks are free in that group (first free read
        // bank from a random start, then a class of it with a free word bank)
        const size_t base = (size_t)g * 32;
        const int s0 = (int)(rng() & 31);
        int rt = -1;
        for (int t = 0; t < 32 && rt < 0; ++t) {
            const int b1 = (s0 + t) & 31;
            if (c1[base + b1]) continue;
            const int q0 = (int)(rng() & 3);
            for (int q = 0; q < 4; ++q) {
                // classes r with r & 31 == b1: r = b1 + 32 * j
                const int r = b1 + 32 * ((q0 + q) & 3);
                if (!c2[base + bank_word(r)] || q == 3) {
                    rt = r;
                    break;
                }
            }
        }
        if (rt < 0) rt = (int)(rng() % NR);
        if (rt == res[a] || of[rt].empty()) continue;
        const int b = of[rt][rng() % of[rt].size()];
        const int ra = res[a];
        int d = move(a, rt);
        d += move(b, ra);
        // accept improvements and sideways moves; rarely an uphill one (a small
        // fixed temperature, deterministic: the generator is seeded)
        if (d <= 0 || u01(rng) < std::exp(-2.0 * d)) {
            swap_pos(a, b);
            cost += d;
            ++accepted;
        } else {
            move(b, rt);
            move(a, ra);
        }
    }
    // labels class by class, columns in ascending id within a class
    std::vector<int> next(NR);
    for (int r = 0; r < NR; ++r) next[r] = r;
    std::vector<std::vector<int>> cols(NR);
    for (int i = 0; i < n; ++i) cols[res[i]].push_back(i);
    // classes may hold more columns than labels of their residue below n
    // (the search keeps class sizes fixed, so this cannot happen; kept exact)
    for (int r = 0; r < NR; ++r)
        for (int c : cols[r]) {
            lab[c] = next[r];
            next[r] += NR;
        }
    if (stats) {
        stats->excess_before = cost0;
        stats->excess_after = total_cost();
        stats->cycles_before = cyc0;
        stats->cycles_after = total_cycles();
        stats->iterations = it;
        stats->accepted = accepted;
    }
    return lab;
}

}  // namespace qldpc
