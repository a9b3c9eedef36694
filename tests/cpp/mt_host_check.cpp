// Host-code self-check of the MT19937 restatement (mt19937.cpp, mt_jump.cpp), built with
// -fsanitize=address,undefined by tests/test_host_sanitizers.py: the one-pass draw against the staged
// draw, the threaded jump-ahead draw against the serial one (shards with odd positions and A = 1..16),
// mt_state_at against stepping.  Exit code 0 = every check held; any sanitizer report aborts.
#include <cstdio>
#include <cstring>
#include <vector>

#include "mt19937.h"

using namespace bcmpc;

static int fails = 0, par_runs = 0;
#define CHECK(c, ...) do { if (!(c)) { std::printf("FAIL: " __VA_ARGS__); std::printf("\n"); ++fails; } } while (0)

static Mt19937 seeded(uint32_t s, int pre) {
    Mt19937 g;
    g.key[0] = s;
    for (int i = 1; i < 624; ++i) g.key[i] = 1812433253u * (g.key[i - 1] ^ (g.key[i - 1] >> 30)) + (uint32_t)i;
    g.pos = 624;
    for (int i = 0; i < pre; ++i) (void)g.next32();
    return g;
}

int main() {
    for (int A : {1, 3, 6, 8, 11, 16})
        for (int pre : {0, 1, 623, 1250}) {
            std::vector<double> lo(A), hi(A);
            for (int j = 0; j < A; ++j) { lo[j] = -1.0 - 0.25 * j; hi[j] = 0.5 + 0.125 * j; }
            const int64_t rows = 3 * 401 + 7;
            // one-pass (all rows kept) against the staged path (keep [0, rows) via two halves)
            Mt19937 g1 = seeded(12345u + A, pre), g2 = g1;
            std::vector<double> a((size_t)rows * A), b((size_t)rows * A);
            mt_uniform_rows(g1, lo.data(), hi.data(), A, rows, 0, rows, a.data());
            const int64_t half = rows / 2;
            Mt19937 g3 = g2;
            mt_uniform_rows(g2, lo.data(), hi.data(), A, half, 0, half, b.data());
            mt_uniform_rows(g2, lo.data(), hi.data(), A, rows - half, 0, rows - half, b.data() + half * A);
            CHECK(std::memcmp(a.data(), b.data(), a.size() * 8) == 0, "one-pass vs split A=%d pre=%d", A, pre);
            CHECK(g1.pos == g2.pos && std::memcmp(g1.key, g2.key, sizeof g1.key) == 0, "state A=%d pre=%d", A, pre);
            // a shard [17, 251) of every 401-row period: staged serial vs the threaded jump-ahead draw
            const int64_t period = 401, klo = 17, khi = 251;
            const int64_t nper = 3, prow = nper * period;      // (the threaded draw takes whole periods)
            std::vector<double> s((size_t)nper * (khi - klo) * A), t(s.size());
            Mt19937 gs = g3, gt = g3;
            for (int64_t p = 0; p < nper; ++p)
                mt_uniform_rows(gs, lo.data(), hi.data(), A, period, klo, khi, s.data() + p * (khi - klo) * A);
            int crc = 0;
            const int used = mt_uniform_rows_par(gt, lo.data(), hi.data(), A, prow, period, klo, khi, t.data(), 3, 256,
                                                 [](int64_t, int64_t) { return 0; }, &crc);
            if (used > 0) {
                ++par_runs;
                CHECK(std::memcmp(s.data(), t.data(), s.size() * 8) == 0, "par vs serial A=%d pre=%d", A, pre);
                CHECK(gs.pos == gt.pos && std::memcmp(gs.key, gt.key, sizeof gs.key) == 0, "par state A=%d", A);
            }
            // mt_state_at against stepping word by word
            Mt19937 gw = g3, gj;
            const int64_t words = 2 * (int64_t)A * rows + 5;
            mt_state_at(g3, words, gj);
            gw.advance(words);
            if (gw.pos >= 624) gw.twist();
            if (gj.pos >= 624) gj.twist();
            CHECK(gw.next32() == gj.next32(), "state_at A=%d pre=%d", A, pre);
        }
    std::printf("%s (%d failures, %d threaded draws compared)\n", fails ? "FAILED" : "ok", fails, par_runs);
    return (fails || par_runs == 0) ? 1 : 0;
}
