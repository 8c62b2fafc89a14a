// java.util.Random (48-bit LCG) batch shuffles for the host runtime: the per-node feature shuffles of
// seriestree/DecisionTree.bagging (reference A/operator/common/tree/seriestree/DecisionTree.java), the same draws
// as common/jrandom.py JavaRandom.shuffle, for a whole tree level in one call instead of ~F Python calls per node.
#include <cstdint>

namespace {

constexpr uint64_t kMult = 0x5DEECE66DULL;
constexpr uint64_t kAdd = 0xBULL;
constexpr uint64_t kMask = (1ULL << 48) - 1;

inline int32_t next_bits(uint64_t& seed, int bits) {
    seed = (seed * kMult + kAdd) & kMask;
    return (int32_t)(uint32_t)(seed >> (48 - bits));
}

inline int32_t next_int(uint64_t& seed, int32_t bound) {
    if ((bound & -bound) == bound) return (int32_t)(((int64_t)bound * (int64_t)next_bits(seed, 31)) >> 31);
    while (true) {
        const int32_t bits = next_bits(seed, 31);
        const int32_t val = bits % bound;
        if ((int32_t)((uint32_t)bits - (uint32_t)val + (uint32_t)(bound - 1)) >= 0) return val;
    }
}

}  // namespace

extern "C" {

// Shuffle m rows of n int32 in place, row after row (Fisher-Yates from the end with nextInt(i + 1), swapping only
// when idx != i), continuing the generator state *seed (the scrambled 48-bit state).
void alink_java_shuffle_rows(uint64_t* seed, int32_t* rows, int64_t m, int32_t n) {
    uint64_t s = *seed;
    for (int64_t r = 0; r < m; ++r) {
        int32_t* a = rows + r * n;
        for (int32_t i = n - 1; i > 0; --i) {
            const int32_t idx = next_int(s, i + 1);
            if (idx == i) continue;
            const int32_t t = a[idx];
            a[idx] = a[i];
            a[i] = t;
        }
    }
    *seed = s;
}

}  // extern "C"
