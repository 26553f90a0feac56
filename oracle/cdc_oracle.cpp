// ORACLE — TEST INFRASTRUCTURE ONLY (see kolm_oracle.cpp's header): never linked into,
// loaded by, or called from the product path.
//
// CPU restatement of the reference's FastCDC chunker, statement by statement:
//   PY:152-165  _make_gear (xorshift32 from 0x243F6A88, entries | 1)
//   PY:172-185  _clamp_mask_bits (bit_length(avg) - 1 clamped to [6, 20])
//   PY:187-193  _roll_gear (fp' = (fp << 1) + GEAR[b] mod 2^32)
//   PY:195-204  _make_low_mask
//   PY:210-309  cdc_fast_boundaries_strict (normalized chunking, orphan-tail merge)
// Pinned by tests/golden/cdc.npz (PY's own boundaries, tests/test_cdc.py).
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace {

std::vector<uint32_t> make_gear(uint32_t seed = 0x243F6A88u) {
    std::vector<uint32_t> t(256);
    uint32_t x = seed;
    for (int i = 0; i < 256; ++i) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        t[i] = x | 1u;
    }
    return t;
}

int clamp_mask_bits(int64_t avg) {
    if (avg <= 0) return 6;
    int k = 63 - __builtin_clzll((uint64_t)avg);  // bit_length - 1
    return k < 6 ? 6 : k > 20 ? 20 : k;
}

uint32_t low_mask(int bits) { return bits <= 0 ? 0u : bits >= 32 ? 0xFFFFFFFFu : (1u << bits) - 1u; }

}  // namespace

extern "C" {

// Chunks of data[0, n) as (start, end) pairs into bounds[2*i], bounds[2*i+1]; returns the
// chunk count, -1 if cap (in pairs) is too small, -2 for the parameter errors PY raises.
int64_t oracle_cdc(const uint8_t* data, int64_t n, int64_t min_size, int64_t avg_size, int64_t max_size,
                   int merge_orphan_tail, int64_t* bounds, int64_t cap) {
    if (n == 0) return 0;
    if (!(min_size > 0 && min_size <= avg_size && avg_size <= max_size)) return -2;
    if (avg_size < 64) return -2;
    static const std::vector<uint32_t> gear = make_gear();
    const int k = clamp_mask_bits(avg_size);
    const int k_str = k + 2 <= 20 ? k + 2 : 20;
    const int k_lo = k > 2 ? k - 2 : 1;
    const uint32_t mask_s = low_mask(k_str), mask_l = low_mask(k_lo);
    std::vector<std::pair<int64_t, int64_t>> b;
    int64_t i = 0;
    while (i < n) {
        const int64_t start = i, remaining = n - start;
        if (remaining <= min_size) {
            b.emplace_back(start, n);
            i = n;
            break;
        }
        const int64_t local_max = remaining < max_size ? remaining : max_size;
        int64_t normal_size = avg_size;
        if (local_max < normal_size) normal_size = local_max;
        const int64_t end_min = start + min_size, end_normal = start + normal_size, end_limit = start + local_max;
        int64_t pos = end_min;
        uint32_t fp = 0;
        bool found = false;
        while (pos < end_normal && pos < end_limit) {
            fp = (fp << 1) + gear[data[pos]];
            if ((fp & mask_s) == 0) {
                pos += 1;
                found = true;
                break;
            }
            pos += 1;
        }
        if (!found) {
            while (pos < end_limit) {
                fp = (fp << 1) + gear[data[pos]];
                if ((fp & mask_l) == 0) {
                    pos += 1;
                    found = true;
                    break;
                }
                pos += 1;
            }
        }
        if (!found) pos = end_limit;
        b.emplace_back(start, pos);
        i = pos;
    }
    if (merge_orphan_tail && b.size() >= 2) {
        const auto last = b.back();
        if (last.second - last.first < min_size) {
            b.pop_back();
            b.back().second = last.second;
        }
    }
    if ((int64_t)b.size() > cap) return -1;
    for (size_t j = 0; j < b.size(); ++j) {
        bounds[2 * j] = b[j].first;
        bounds[2 * j + 1] = b[j].second;
    }
    return (int64_t)b.size();
}

}  // extern "C"
