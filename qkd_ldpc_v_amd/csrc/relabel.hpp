// relabel.hpp — bank-aware relabelling of bit ids (relabel.cpp; host only).
#pragma once
#include <cstdint>
#include <vector>

namespace qldpc {

// One member of an LDS access group: a column (bit id) or, col < 0, a fixed
// address of class fixed_res (the dummy column n of padding slots); fmask bit 0:
// the member takes part in the 64-bit total read (bank = class mod 32), bit 1:
// in the code-word OR (bank = (class >> 2) mod 32).
struct RelabelMember {
    int32_t col;
    int32_t fixed_res;
    uint8_t fmask;
};
// The lanes of one wave half that access LDS together (one slot of the layout).
struct RelabelGroup {
    std::vector<RelabelMember> members;
};
struct RelabelStats {
    long long excess_before = 0, excess_after = 0;  // summed max(0, count - 1) over groups and banks
    long long cycles_before = 0, cycles_after = 0;  // summed busiest-bank count over groups (LDS cycles per half)
    long long iterations = 0, accepted = 0;
};

// lab[orig] = new label (a permutation of 0..n-1).  Deterministic for a seed.
std::vector<int32_t> bank_relabel(int n, const std::vector<RelabelGroup> &groups, uint64_t seed, long long iters,
                                  RelabelStats *stats);

}  // namespace qldpc
