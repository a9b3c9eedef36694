// mt19937.h -- the legacy NumPy global generator on the host (internal to libbcmpc).
//
// MPCcontroller.sample_random_actions (controllers.py:43-55) draws
// np.random.uniform(low, high, [H, K, A]) from NumPy's legacy RandomState:
// MT19937 (Matsumoto & Nishimura 1998; NumPy's randomkit twist, mt19937.c) and
// random_sample = ((w1 >> 5) * 2^26 + (w2 >> 6)) / 2^53 from two tempered words,
// then uniform = low + (high - low) * d in f64 (mul, then add: no FMA).  This
// restatement continues the stream from NumPy's own state (np.random.get_state())
// and returns the advanced state, so the caller's global stream moves exactly as
// one np.random.uniform call would move it.
#pragma once
#include <stdint.h>

#include <functional>
#include <vector>

namespace bcmpc {

struct Mt19937 {
    uint32_t key[624];
    int32_t pos;

    void twist() {
        constexpr uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kMatrix = 0x9908b0dfu;
        int i = 0;
        for (; i < 624 - 397; ++i) {
            const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + 397] ^ (y >> 1) ^ (-(y & 1u) & kMatrix);
        }
        for (; i < 623; ++i) {
            const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + 397 - 624] ^ (y >> 1) ^ (-(y & 1u) & kMatrix);
        }
        const uint32_t y = (key[623] & kUpper) | (key[0] & kLower);
        key[623] = key[396] ^ (y >> 1) ^ (-(y & 1u) & kMatrix);
        pos = 0;
    }
    uint32_t next32() {
        if (pos >= 624) twist();
        uint32_t y = key[pos++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
    // skip n raw words: the state n next32() calls leave behind (no tempering, nothing stored)
    void advance(int64_t n) {
        while (n > 0) {
            if (pos >= 624) twist();
            const int64_t take = n < 624 - pos ? n : 624 - pos;
            pos += (int32_t)take;
            n -= take;
        }
    }
    double next_double() {
        const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
        return (a * 67108864.0 + b) / 9007199254740992.0;
    }
};

// n_rows rows of A uniforms (C order): out[r * A + j] = low[j] + (high[j] - low[j]) * d.
// Rows outside [keep_lo, keep_hi) are drawn (the stream advances) but not stored; kept row r
// lands at out[(r - keep_lo) * A + j].
void mt_uniform_rows(Mt19937& g, const double* low, const double* high, int A, int64_t n_rows, int64_t keep_lo,
                     int64_t keep_hi, double* out);

// the next m random_sample doubles of the stream
void mt_next_doubles(Mt19937& g, double* dbl, int64_t m);

// ---- jump-ahead (mt_jump.cpp) ----
// BCMPC_MT_THREADS, else min(8, hardware threads)
int mt_default_threads();
// out = the state at the start of block `blocks` (>= 1) after g's key block: key = that block's
// 624 raw words, pos = 0 (the words twist(g.key) would hold after `blocks` twists)
void mt_jump_blocks(const Mt19937& g, int64_t blocks, Mt19937& out);
// x^(624 (f - 1)) mod phi for each f (>= 1; the jump from a stream's block 1 to its block f), packed
// as 624 u32 words per polynomial (bit i % 32 of word i / 32 = coefficient of x^i); cached per process
void mt_block_polys(const std::vector<int64_t>& fs, uint32_t* out);
// out = g advanced by `words` generator words (a jump to the block that holds the word, then its position)
void mt_state_at(const Mt19937& g, int64_t words, Mt19937& out);
// The same draw as mt_uniform_rows over n_rows rows, for a keep set that repeats with `period` rows:
// row r is kept iff r % period is in [keep_lo, keep_hi) and lands at output row
// (r / period) * (keep_hi - keep_lo) + r % period - keep_lo.  The kept rows are split over up to
// `threads` host threads (each >= min_words_per_thread generator words); a thread jumps to the start
// of every run of kept rows it draws, so a shard's draw costs its own rows plus one jump per run, not
// the whole stream.  Each thread hands its output on in ranges [o_lo, o_hi) (doubles, ~2 MiB each)
// to on_chunk as they are written (from that thread, in order); the first nonzero on_chunk result
// lands in *chunk_rc.  Returns the number of threads used, or 0 (nothing drawn) when the kept draw
// is too small to split; g ends exactly where NumPy's one draw of all n_rows rows leaves it.
int mt_uniform_rows_par(Mt19937& g, const double* low, const double* high, int A, int64_t n_rows, int64_t period,
                         int64_t keep_lo, int64_t keep_hi, double* out, int threads, int64_t min_words_per_thread,
                         const std::function<int(int64_t, int64_t)>& on_chunk, int* chunk_rc);

}  // namespace bcmpc
