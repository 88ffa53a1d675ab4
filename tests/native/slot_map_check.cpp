// Host check of the payload slot map (csrc/pd_common.h term_slot / slot_of_pair): for every way
// of splitting 50 neighbourhood points over the five AoA columns, the 50 terms fill the 25 pair
// slots' 50 positions exactly once, a non-general slot holds two consecutive points of one
// column window, and a cross slot (two odd windows' last points) sits in a general position.
#include "pd_common.h"
#include <cstdio>
using namespace pd;
int main() {
    long bad = 0, combos = 0;
    int len[kCols];
    for (len[0] = 0; len[0] <= kNbr; ++len[0])
    for (len[1] = 0; len[0] + len[1] <= kNbr; ++len[1])
    for (len[2] = 0; len[0] + len[1] + len[2] <= kNbr; ++len[2])
    for (len[3] = 0; len[0] + len[1] + len[2] + len[3] <= kNbr; ++len[3]) {
        len[4] = kNbr - len[0] - len[1] - len[2] - len[3];
        ++combos;
        int used[2 * kPairs] = {0}, col_of[2 * kPairs], off_of[2 * kPairs];
        int t = 0;
        for (int c = 0; c < kCols; ++c)
            for (int i = 0; i < len[c]; ++i, ++t) {
                int k, p;
                term_slot(len, t, k, p);
                if (k < 0 || k >= kPairs || p < 0 || p > 1) { ++bad; continue; }
                used[2 * k + p]++;
                col_of[2 * k + p] = c;
                off_of[2 * k + p] = i;
            }
        for (int j = 0; j < 2 * kPairs; ++j) if (used[j] != 1) { ++bad; break; }
        if (bad) continue;
        for (int k = 0; k < kPairs; ++k) {
            const bool same = col_of[2 * k] == col_of[2 * k + 1] && off_of[2 * k + 1] == off_of[2 * k] + 1;
            if (!slot_general(k) && !same) ++bad;          // (p, p + 1) of one window
            if (!same) {                                   // cross slot: both odd windows' last points
                const int c0 = col_of[2 * k], c1 = col_of[2 * k + 1];
                if (!(len[c0] & 1) || !(len[c1] & 1) || off_of[2 * k] != len[c0] - 1 || off_of[2 * k + 1] != len[c1] - 1) ++bad;
            }
        }
    }
    std::printf("combos %ld bad %ld\n", combos, bad);
    return bad != 0;
}
