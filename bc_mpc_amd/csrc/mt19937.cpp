// mt19937.cpp -- bulk uniforms from NumPy's legacy MT19937 stream (see mt19937.h).
#include "mt19937.h"

#include <algorithm>
#include <vector>

namespace bcmpc {

namespace {

inline uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

}  // namespace

// the next m random_sample doubles of the stream (mt19937_next_double, two words each);
// AVX-512 / AVX2 clones where the host has them (same integer ops and exactly rounded conversions)
__attribute__((target_clones("avx512f", "avx2", "default")))
void mt_next_doubles(Mt19937& g, double* dbl, int64_t m) {
    int64_t i = 0;
    while (i < m) {
        if (g.pos >= 624) g.twist();
        const int avail = 624 - g.pos;
        if (avail >= 2) {
            const int64_t nd = std::min<int64_t>(avail / 2, m - i);
            const uint32_t* w = g.key + g.pos;
            double* o = dbl + i;
            for (int64_t k = 0; k < nd; ++k) {      // vectorisable: no cross-iteration state
                const uint32_t a = temper(w[2 * k]) >> 5, b = temper(w[2 * k + 1]) >> 6;
                o[k] = ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);   // / 2^53, exact
            }
            g.pos += (int32_t)(2 * nd);
            i += nd;
        } else {                                    // one word left: the double straddles the twist
            const uint32_t a = temper(g.key[623]) >> 5;
            g.twist();
            const uint32_t b = temper(g.key[0]) >> 6;
            g.pos = 1;
            dbl[i++] = ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
        }
    }
}

// The next m uniforms of a row-major [.][A] draw, low[j] + range[j] * d (random_uniform: mul, then add)
// with d the next random_sample double, written straight into out (one pass: tempering, the exact
// double and the scaling vectorise together).  pl / pr: the per-column bounds repeated over 2 Lp entries
// (Lp = lcm(A, 8) doubles, a whole number of SIMD vectors); the column of out[0] is column 0.
__attribute__((target_clones("avx512f", "avx2", "default")))
static void mt_uniform_flat(Mt19937& g, const double* pl, const double* pr, int Lp, double* out, int64_t m) {
    int64_t i = 0;
    while (i < m) {
        if (g.pos >= 624) g.twist();
        const int avail = 624 - g.pos;
        if (avail >= 2) {
            const int64_t nd = std::min<int64_t>(avail / 2, m - i);
            const uint32_t* w = g.key + g.pos;
            int64_t k = 0;
            const int t0 = (int)(i % Lp);
            for (; k + Lp <= nd; k += Lp) {                // whole pattern periods: vectorisable
                double* o = out + i + k;
                const uint32_t* ww = w + 2 * k;
                const double* lo = pl + t0;
                const double* rg = pr + t0;
                for (int t = 0; t < Lp; ++t) {
                    const uint32_t a = temper(ww[2 * t]) >> 5, b = temper(ww[2 * t + 1]) >> 6;
                    const double d = ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
                    o[t] = lo[t] + rg[t] * d;
                }
            }
            for (; k < nd; ++k) {
                const uint32_t a = temper(w[2 * k]) >> 5, b = temper(w[2 * k + 1]) >> 6;
                const double d = ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
                const int t = (int)((i + k) % Lp);
                out[i + k] = pl[t] + pr[t] * d;
            }
            g.pos += (int32_t)(2 * nd);
            i += nd;
        } else {                                    // one word left: the double straddles the twist
            const uint32_t a = temper(g.key[623]) >> 5;
            g.twist();
            const uint32_t b = temper(g.key[0]) >> 6;
            g.pos = 1;
            const int t = (int)(i % Lp);
            out[i] = pl[t] + pr[t] * (((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0));
            ++i;
        }
    }
}

void mt_uniform_rows(Mt19937& g, const double* low, const double* high, int A, int64_t n_rows, int64_t keep_lo,
                     int64_t keep_hi, double* out) {
    if (keep_lo <= 0 && keep_hi >= n_rows && A <= 16) {
        // every row kept: one pass into out (the bound patterns on the stack: Lp <= 128 doubles)
        int Lp = A;
        while (Lp % 8) Lp += A;
        double pl[256], pr[256];
        for (int t = 0; t < 2 * Lp; ++t) {
            pl[t] = low[t % A];
            pr[t] = high[t % A] - low[t % A];                  // np.subtract(high, low)
        }
        mt_uniform_flat(g, pl, pr, Lp, out, n_rows * A);
        return;
    }
    std::vector<double> range((size_t)A);                      // (any A: no fixed-size buffer)
    for (int j = 0; j < A; ++j) range[j] = high[j] - low[j];    // np.subtract(high, low)
    constexpr int64_t kRows = 2048;
    double buf[kRows * 16];
    const int64_t rows_per = std::max<int64_t>(1, (int64_t)(sizeof(buf) / sizeof(double)) / A);
    for (int64_t r0 = 0; r0 < n_rows; r0 += rows_per) {
        const int64_t nr = std::min(rows_per, n_rows - r0);
        mt_next_doubles(g, buf, nr * A);
        const int64_t a = std::max(r0, keep_lo), b = std::min(r0 + nr, keep_hi);
        for (int64_t r = a; r < b; ++r) {
            const double* d = buf + (r - r0) * A;
            double* o = out + (r - keep_lo) * A;
            for (int j = 0; j < A; ++j) o[j] = low[j] + range[j] * d[j];   // random_uniform: mul, then add
        }
    }
}

}  // namespace bcmpc
