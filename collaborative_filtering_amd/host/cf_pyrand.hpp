// cf_pyrand.hpp -- CPython's random.Random (MT19937) restated, so that
// bin/fold_cross_validation shuffles the users exactly as fold_cross_validation.py:38
// (`random.shuffle(keys)`) does after `random.seed(S)`:
//   random.seed(int)          -> init_by_array over the 32-bit words of |S| (_randommodule.c)
//   getrandbits(k), k <= 32   -> genrand_uint32() >> (32 - k)
//   _randbelow(n)             -> getrandbits(n.bit_length()) until < n (random.py)
//   shuffle(x)                -> for i = len-1 .. 1: j = _randbelow(i + 1); swap (random.py)
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace pyrand {

class MT {
    uint32_t mt[624];
    int mti = 625;

    void init_genrand(uint32_t s) {
        mt[0] = s;
        for (mti = 1; mti < 624; ++mti) mt[mti] = 1812433253u * (mt[mti - 1] ^ (mt[mti - 1] >> 30)) + (uint32_t)mti;
    }

public:
    explicit MT(uint64_t seed) {   // random.seed(seed) for a non-negative int
        std::vector<uint32_t> key;
        do {
            key.push_back((uint32_t)seed);
            seed >>= 32;
        } while (seed);
        init_genrand(19650218u);
        uint32_t i = 1, j = 0;
        const uint32_t len = (uint32_t)key.size();
        for (uint32_t k = 624 > len ? 624 : len; k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + j;
            ++i;
            ++j;
            if (i >= 624) {
                mt[0] = mt[623];
                i = 1;
            }
            if (j >= len) j = 0;
        }
        for (uint32_t k = 623; k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - i;
            ++i;
            if (i >= 624) {
                mt[0] = mt[623];
                i = 1;
            }
        }
        mt[0] = 0x80000000u;
        mti = 624;
    }

    uint32_t genrand_uint32() {
        static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
        if (mti >= 624) {
            int kk = 0;
            for (; kk < 624 - 397; ++kk) {
                const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
            }
            for (; kk < 623; ++kk) {
                const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
            }
            const uint32_t y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
            mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
            mti = 0;
        }
        uint32_t y = mt[mti++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }

    // _randbelow_with_getrandbits for 0 < n < 2^32
    uint32_t randbelow(uint32_t n) {
        int k = 0;
        while (k < 32 && (n >> k)) ++k;   // n.bit_length()
        uint32_t r = genrand_uint32() >> (32 - k);
        while (r >= n) r = genrand_uint32() >> (32 - k);
        return r;
    }

    template <class T>
    void shuffle(std::vector<T>& x) {
        for (size_t i = x.size(); i-- > 1;) {
            const size_t j = randbelow((uint32_t)(i + 1));
            std::swap(x[i], x[j]);
        }
    }
};

}  // namespace pyrand
