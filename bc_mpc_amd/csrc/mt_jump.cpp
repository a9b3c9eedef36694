// mt_jump.cpp -- NumPy's legacy MT19937 stream drawn by several host threads (see mt19937.h).
//
// The generator's words obey x[k+624] = x[k+397] ^ mix(x[k], x[k+1]), a linear map F on the
// 624-word window W_k = (x[k] .. x[k+623]) over GF(2).  On every window the generator can reach
// (the image of F) the characteristic polynomial phi (degree 19937) annihilates F, so
// F^J W = (x^J mod phi)(F) W  (Haramoto, Matsumoto, L'Ecuyer 2008, "A fast jump ahead algorithm for
// linear recurrences in a polynomial space").  phi is found once per process by Berlekamp-Massey on
// one bit of the generated words; x^J mod phi by square-and-multiply; the polynomial is applied to a
// window by Horner's rule (one generator step per coefficient, one window XOR per set coefficient).
//
// Thread t >= 1 starts at a block boundary b0 + 624 * t * M of the caller's stream (b0 = the caller's
// key block), so its start window is F^(624 (tM - 1)) applied to twist(key) and the jump polynomials
// depend only on (t, M): they are cached per process.  Thread t draws the doubles that start in its
// blocks; the last thread ends in exactly the (key, pos) NumPy itself would hold.
#include "mt19937.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include <emmintrin.h>
#include <smmintrin.h>
#include <wmmintrin.h>

namespace bcmpc {

namespace {

constexpr int kDeg = 19937;                   // degree of MT19937's characteristic polynomial
constexpr int kPW = kDeg / 64 + 1;            // words of a polynomial of degree <= kDeg
constexpr int kN = 624, kM = 397;
using Poly = std::vector<uint64_t>;

inline uint32_t mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
}
inline int bit(const uint64_t* p, int64_t i) { return (int)((p[i >> 6] >> (i & 63)) & 1u); }

// r ^= p << s (p: np words)
void xor_shifted(uint64_t* r, const uint64_t* p, int np, int64_t s) {
    const int64_t ws = s >> 6;
    const int bs = (int)(s & 63);
    if (bs == 0) {
        for (int w = 0; w < np; ++w) r[w + ws] ^= p[w];
    } else {
        for (int w = 0; w < np; ++w) {
            r[w + ws] ^= p[w] << bs;
            r[w + ws + 1] ^= p[w] >> (64 - bs);
        }
    }
}

// Berlekamp-Massey over GF(2) on the LSBs of generated words; returns phi (bit i = coeff of x^i)
Poly compute_phi() {
    Mt19937 g;
    g.key[0] = 5489u;                                      // init_genrand(5489)
    for (int i = 1; i < kN; ++i) g.key[i] = 1812433253u * (g.key[i - 1] ^ (g.key[i - 1] >> 30)) + (uint32_t)i;
    g.pos = kN;
    const int64_t N = 2 * (int64_t)kDeg + 128;
    std::vector<uint8_t> s((size_t)N);
    for (int64_t n = 0; n < N; ++n) {
        if (g.pos >= kN) g.twist();                        // raw (untempered) words, all generated
        s[(size_t)n] = (uint8_t)(g.key[g.pos++] & 1u);
    }
    const int NW = (int)(N / 64) + 2;
    Poly C(NW, 0), B(NW, 0), T(NW, 0), R(NW, 0);
    C[0] = B[0] = 1;
    int L = 0;
    int64_t m = 1;
    for (int64_t n = 0; n < N; ++n) {
        // R bit i = s[n - i]
        for (int w = NW - 1; w > 0; --w) R[w] = (R[w] << 1) | (R[w - 1] >> 63);
        R[0] = (R[0] << 1) | s[(size_t)n];
        const int lw = L / 64 + 1;
        uint64_t acc = 0;
        for (int w = 0; w < lw; ++w) acc ^= C[w] & R[w];
        const int d = __builtin_popcountll(acc) & 1;
        if (!d) {
            ++m;
        } else if (2 * L <= n) {
            T = C;
            xor_shifted(C.data(), B.data(), (int)(NW - 1 - (m >> 6)), m);
            L = (int)(n + 1 - L);
            B = T;
            m = 1;
        } else {
            xor_shifted(C.data(), B.data(), (int)(NW - 1 - (m >> 6)), m);
            ++m;
        }
    }
    if (L != kDeg) std::abort();                           // MT19937's recurrence has degree 19937
    Poly phi(kPW, 0);                                      // phi(x) = x^L C(1/x)
    for (int i = 0; i <= L; ++i)
        if (bit(C.data(), i)) phi[(size_t)(L - i) >> 6] |= 1ull << ((L - i) & 63);
    return phi;
}

const Poly& phi_poly() {
    static const Poly phi = compute_phi();
    return phi;
}

// r = a * b (carry-less), r: 2 * kPW + 1 words, zeroed by the caller
__attribute__((target("pclmul,sse4.1")))
void clmul_poly_hw(const uint64_t* a, const uint64_t* b, uint64_t* r) {
    for (int i = 0; i < kPW; ++i) {
        if (!a[i]) continue;
        const __m128i ai = _mm_set_epi64x(0, (long long)a[i]);
        for (int j = 0; j < kPW; ++j) {
            const __m128i p = _mm_clmulepi64_si128(ai, _mm_set_epi64x(0, (long long)b[j]), 0x00);
            r[i + j] ^= (uint64_t)_mm_cvtsi128_si64(p);
            r[i + j + 1] ^= (uint64_t)_mm_extract_epi64(p, 1);
        }
    }
}

void clmul_poly_sw(const uint64_t* a, const uint64_t* b, uint64_t* r) {
    for (int64_t i = 0; i < kDeg; ++i)
        if (bit(a, i)) xor_shifted(r, b, kPW, i);
}

void clmul_poly(const uint64_t* a, const uint64_t* b, uint64_t* r) {
    static const bool hw = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    if (hw) clmul_poly_hw(a, b, r);
    else clmul_poly_sw(a, b, r);
}

// the kPW low words of r >> s (r: nw words)
Poly shr(const uint64_t* r, int nw, int64_t s) {
    Poly o(kPW, 0);
    const int64_t ws = s >> 6;
    const int bs = (int)(s & 63);
    for (int w = 0; w < kPW; ++w) {
        const int64_t i = w + ws;
        const uint64_t lo = i < nw ? r[i] : 0, hi = i + 1 < nw ? r[i + 1] : 0;
        o[w] = bs ? (lo >> bs) | (hi << (64 - bs)) : lo;
    }
    return o;
}

// Barrett constant mu = floor(x^(2 kDeg) / phi) (degree kDeg), by long division once per process
const Poly& barrett_mu() {
    static const Poly mu = [] {
        const Poly& phi = phi_poly();
        Poly rem(2 * kPW + 1, 0), q(kPW, 0);
        rem[(2 * kDeg) >> 6] |= 1ull << ((2 * kDeg) & 63);
        for (int64_t i = 2 * (int64_t)kDeg; i >= kDeg; --i)
            if (bit(rem.data(), i)) {
                q[(size_t)(i - kDeg) >> 6] |= 1ull << ((i - kDeg) & 63);
                xor_shifted(rem.data(), phi.data(), kPW, i - kDeg);
            }
        return q;
    }();
    return mu;
}

// r (2 kPW + 1 words, deg < 2 kDeg) mod phi into out (kPW words) by Barrett reduction:
// q = ((r >> n) mu) >> n, out = r - q phi (exact over GF(2)); ~10x faster than the bitwise reduce
void barrett_reduce(const uint64_t* r, uint64_t* out) {
    const Poly& phi = phi_poly();
    const Poly& mu = barrett_mu();
    Poly t(2 * kPW + 1, 0), u(2 * kPW + 1, 0);
    const Poly rh = shr(r, 2 * kPW + 1, kDeg);
    clmul_poly(rh.data(), mu.data(), t.data());
    const Poly q = shr(t.data(), 2 * kPW + 1, kDeg);
    clmul_poly(q.data(), phi.data(), u.data());
    for (int w = 0; w < kPW; ++w) out[w] = r[w] ^ u[w];
    out[kPW - 1] &= (1ull << (kDeg & 63)) - 1;        // bits >= kDeg cancel exactly
}

// a * b mod phi
Poly mulmod(const Poly& a, const Poly& b) {
    Poly r(2 * kPW + 1, 0), out(kPW, 0);
    clmul_poly(a.data(), b.data(), r.data());
    barrett_reduce(r.data(), out.data());
    return out;
}

// x^e mod phi
Poly x_pow_mod(uint64_t e) {
    const Poly& phi = phi_poly();
    static const uint16_t* spread = [] {
        static uint16_t t[256];
        for (int b = 0; b < 256; ++b) {
            uint16_t v = 0;
            for (int k = 0; k < 8; ++k) v |= (uint16_t)(((b >> k) & 1) << (2 * k));
            t[b] = v;
        }
        return t;
    }();
    Poly r(2 * kPW + 1, 0), sq(2 * kPW + 1, 0);
    r[0] = 1;
    for (int b = 63; b >= 0; --b) {
        if ((e >> b) == 0) continue;                       // leading zeros
        // r = r^2 mod phi
        std::fill(sq.begin(), sq.end(), 0);
        for (int w = 0; w < kPW; ++w) {
            const uint64_t v = r[w];
            uint64_t lo = 0, hi = 0;
            for (int k = 0; k < 4; ++k) lo |= (uint64_t)spread[(v >> (8 * k)) & 255] << (16 * k);
            for (int k = 0; k < 4; ++k) hi |= (uint64_t)spread[(v >> (32 + 8 * k)) & 255] << (16 * k);
            sq[2 * w] = lo;
            sq[2 * w + 1] = hi;
        }
        barrett_reduce(sq.data(), r.data());
        std::fill(r.begin() + kPW, r.end(), 0);
        if ((e >> b) & 1u) {                               // r = r * x mod phi
            for (int w = kPW; w > 0; --w) r[w] = (r[w] << 1) | (r[w - 1] >> 63);
            r[0] <<= 1;
            if (bit(r.data(), kDeg)) xor_shifted(r.data(), phi.data(), kPW, 0);
        }
    }
    r.resize(kPW);
    return r;
}

// cached x^(624 * blocks) mod phi
const Poly& block_jump(int64_t blocks) {
    static std::mutex mu;
    static std::map<int64_t, Poly> cache;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(blocks);
        if (it != cache.end()) return it->second;
    }
    Poly p = x_pow_mod((uint64_t)blocks * kN);
    std::lock_guard<std::mutex> lk(mu);
    return cache.emplace(blocks, std::move(p)).first->second;   // (std::map nodes never move)
}

// out = g(F) w  (w a reachable window).  Horner over 8-coefficient blocks (the sliding-window
// form of Haramoto et al.): tab[v] = sum_j v_j F^j w for every byte v (F^j w = w's stream shifted by
// j words), then acc = F^8 acc ^ tab[block] from the top block down: one window XOR per 8
// coefficients instead of one per set coefficient.
__attribute__((target_clones("avx2", "default")))
void apply_poly(const Poly& g, const uint32_t* w, uint32_t* out) {
    constexpr int kQ = 8;
    std::vector<uint32_t> ext(kN + kQ);                    // w's stream: x[0 .. 624 + kQ)
    std::memcpy(ext.data(), w, kN * sizeof(uint32_t));
    for (int k = kN; k < kN + kQ; ++k) ext[k] = ext[k - kN + kM] ^ mix(ext[k - kN], ext[k - kN + 1]);
    std::vector<uint32_t> tab((size_t)(1 << kQ) * kN);
    std::memset(tab.data(), 0, kN * sizeof(uint32_t));
    for (int v = 1; v < (1 << kQ); ++v) {
        const int top = 31 - __builtin_clz((unsigned)v);
        const uint32_t* a = tab.data() + (size_t)(v ^ (1 << top)) * kN;
        const uint32_t* b = ext.data() + top;
        uint32_t* d = tab.data() + (size_t)v * kN;
        for (int j = 0; j < kN; ++j) d[j] = a[j] ^ b[j];
    }
    std::vector<uint32_t> buf(2 * kN, 0);
    uint32_t* acc = buf.data();
    int s = 0;
    const int nblk = (kDeg + kQ - 1) / kQ;
    bool started = false;
    for (int blk = nblk - 1; blk >= 0; --blk) {
        unsigned v = 0;
        for (int j = 0; j < kQ; ++j) {
            const int i = blk * kQ + j;
            if (i < kDeg && bit(g.data(), i)) v |= 1u << j;
        }
        if (started) {
            for (int k = 0; k < kQ; ++k) {                  // acc = F^8 acc
                acc[s + kN] = acc[s + kM] ^ mix(acc[s], acc[s + 1]);
                if (++s == kN) {
                    std::memcpy(acc, acc + kN, kN * sizeof(uint32_t));
                    s = 0;
                }
            }
        }
        if (v) {
            const uint32_t* t = tab.data() + (size_t)v * kN;
            uint32_t* a = acc + s;
            for (int j = 0; j < kN; ++j) a[j] ^= t[j];
            started = true;
        }
    }
    std::memcpy(out, acc + s, kN * sizeof(uint32_t));
}

// cached x^(624 (f - 1)) mod phi: the jump from block 1 to block f of a stream (f >= 1)
std::mutex g_fpoly_mu;
std::map<int64_t, Poly> g_fpoly;

}  // namespace

void mt_block_polys(const std::vector<int64_t>& fs, uint32_t* out) {
    std::vector<int64_t> want;
    {
        std::lock_guard<std::mutex> lk(g_fpoly_mu);
        for (int64_t f : fs)
            if (f >= 1 && !g_fpoly.count(f)) want.push_back(f);
    }
    std::sort(want.begin(), want.end());
    want.erase(std::unique(want.begin(), want.end()), want.end());
    if (!want.empty()) {
        // sorted runs per thread: the run's first polynomial by square-and-multiply, the rest by one
        // multiplication each with the (cached) step polynomial x^(624 (f_i - f_{i-1}))
        const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)mt_default_threads(), (want.size() + 7) / 8));
        for (int t = 0; t < T; ++t) {                    // the steps every run uses, once
            const size_t a = want.size() * t / T, b = want.size() * (t + 1) / T;
            for (size_t i = a + 1; i < b; ++i) (void)block_jump(want[i] - want[i - 1]);
        }
        std::vector<Poly> res(want.size());
        auto work = [&](int t) {
            const size_t a = want.size() * t / T, b = want.size() * (t + 1) / T;
            for (size_t i = a; i < b; ++i) {
                if (i == a) res[i] = x_pow_mod((uint64_t)kN * (uint64_t)(want[i] - 1));
                else res[i] = mulmod(res[i - 1], block_jump(want[i] - want[i - 1]));
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
        work(0);
        for (auto& th : pool) th.join();
        std::lock_guard<std::mutex> lk(g_fpoly_mu);
        for (size_t i = 0; i < want.size(); ++i) g_fpoly.emplace(want[i], std::move(res[i]));
    }
    std::lock_guard<std::mutex> lk(g_fpoly_mu);
    for (size_t k = 0; k < fs.size(); ++k) {
        const Poly& p = g_fpoly.at(std::max<int64_t>(1, fs[k]));
        uint32_t* o = out + k * 624;
        for (int w = 0; w < 312; ++w) {
            o[2 * w] = (uint32_t)p[w];
            o[2 * w + 1] = (uint32_t)(p[w] >> 32);
        }
    }
}

int mt_default_threads() {
    const char* e = std::getenv("BCMPC_MT_THREADS");
    if (e && *e) return std::max(1, std::atoi(e));
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::min<unsigned>(8u, hc ? hc : 1u);
}

void mt_jump_blocks(const Mt19937& g, int64_t blocks, Mt19937& out) {
    // W1 = twist(key): the window one block past the caller's key block (generated, so reachable)
    Mt19937 t = g;
    t.twist();
    if (blocks <= 1) {
        out = t;
    } else {
        apply_poly(block_jump(blocks - 1), t.key, out.key);
    }
    out.pos = 0;
}

void mt_state_at(const Mt19937& g, int64_t words, Mt19937& out) {
    const int64_t p = g.pos + words;                     // word index relative to g's key block
    const int64_t f = p / kN;
    if (f == 0) {
        out = g;
    } else {
        mt_jump_blocks(g, f, out);
    }
    out.pos = (int32_t)(p - f * kN);
}

int mt_uniform_rows_par(Mt19937& g, const double* low, const double* high, int A, int64_t n_rows, int64_t period,
                        int64_t keep_lo, int64_t keep_hi, double* out, int threads, int64_t min_words_per_thread,
                        const std::function<int(int64_t, int64_t)>& on_chunk, int* chunk_rc) {
    if (period < 1 || n_rows % period || keep_lo < 0 || keep_hi > period || keep_lo >= keep_hi) return 0;
    const int64_t nper = n_rows / period, kw = keep_hi - keep_lo;
    const int64_t rows_k = nper * kw;                    // kept rows (= output rows)
    const int64_t words_k = 2 * rows_k * A;              // generator words behind them
    int T = threads;
    if (min_words_per_thread > 0) T = (int)std::min<int64_t>(T, words_k / min_words_per_thread);
    T = (int)std::min<int64_t>(T, rows_k);
    if (T < 2) return 0;
    // kept runs of global rows [r0, r1) -> output rows from o0 (one run per period, merged when
    // they touch: a whole-draw keep is one run); every thread jumps to the start of each run it
    // touches, so a shard draws only its own rows (plus one jump per run)
    struct Run { int64_t r0, r1, o0; };
    std::vector<Run> runs;
    for (int64_t p = 0; p < nper; ++p) {
        const int64_t r0 = p * period + keep_lo, r1 = p * period + keep_hi;
        if (!runs.empty() && runs.back().r1 == r0) runs.back().r1 = r1;
        else runs.push_back({r0, r1, p * kw});
    }
    std::vector<double> range((size_t)A);
    for (int j = 0; j < A; ++j) range[j] = high[j] - low[j];   // np.subtract(high, low)
    constexpr int64_t kRows = 1024, kFlush = int64_t(1) << 18;   // rows per generator call; doubles
    std::vector<double> lowx((size_t)(kRows * A)), rangex((size_t)(kRows * A));
    for (int64_t i = 0; i < kRows * A; ++i) { lowx[i] = low[i % A]; rangex[i] = range[i % A]; }
    std::vector<Mt19937> gs(T);
    std::vector<int64_t> last_end(T, -1);                 // global row each thread's generator stopped at
    std::vector<int> rcs(T, 0);
    static const bool dbg = std::getenv("BCMPC_MT_DEBUG") != nullptr;
    auto work = [&](int t) {
        const auto t0 = std::chrono::steady_clock::now();
        double jump_ms = 0.0;
        const int64_t oa = rows_k * t / T, ob = rows_k * (t + 1) / T;   // this thread's output rows
        std::vector<double> bufv((size_t)(kRows * A));
        double* buf = bufv.data();
        Mt19937& gt = gs[t];
        int64_t at = -1;                                   // global row gt is positioned at
        int64_t o_lo = -1, o_hi = -1;                      // output doubles written, not yet handed on
        // first run holding output row oa
        size_t ri = (size_t)(std::upper_bound(runs.begin(), runs.end(), oa,
                                              [](int64_t o, const Run& r) { return o < r.o0; }) - runs.begin()) - 1;
        for (int64_t o = oa; o < ob; ++ri) {
            const Run& r = runs[ri];
            const int64_t g0 = r.r0 + (o - r.o0);
            const int64_t n_rows_here = std::min(ob - o, (r.r1 - r.r0) - (o - r.o0));
            if (at != g0) {
                const auto j0 = std::chrono::steady_clock::now();
                mt_state_at(g, 2 * g0 * A, gt);
                jump_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - j0).count();
            }
            for (int64_t done = 0; done < n_rows_here;) {
                const int64_t nr = std::min(kRows, n_rows_here - done);
                const int64_t n = nr * A;
                mt_next_doubles(gt, buf, n);
                double* dst = out + (o + done) * A;
                const double* lx = lowx.data();
                const double* rx = rangex.data();
                int64_t i = 0;
                if (((uintptr_t)dst & 15) && n > 0) { dst[0] = lx[0] + rx[0] * buf[0]; i = 1; }
                // streaming stores: the output is read next by the DMA engine, not by this core
                for (; i + 2 <= n; i += 2)
                    _mm_stream_pd(dst + i, _mm_add_pd(_mm_loadu_pd(lx + i), _mm_mul_pd(_mm_loadu_pd(rx + i),
                                                                                       _mm_loadu_pd(buf + i))));
                for (; i < n; ++i) dst[i] = lx[i] + rx[i] * buf[i];   // random_uniform: mul, then add
                if (o_lo < 0) o_lo = (o + done) * A;
                o_hi = (o + done + nr) * A;
                done += nr;
                // hand finished output on in ~2 MiB pieces, so its copy overlaps the rest of the draw
                if (on_chunk && o_hi - o_lo >= kFlush && !rcs[t]) {
                    _mm_sfence();
                    rcs[t] = on_chunk(o_lo, o_hi);
                    o_lo = -1;
                }
            }
            o += n_rows_here;
            at = g0 + n_rows_here;
        }
        _mm_sfence();                                      // streaming stores visible before any copy
        if (on_chunk && o_lo >= 0 && !rcs[t]) rcs[t] = on_chunk(o_lo, o_hi);
        last_end[t] = at;
        if (dbg) {
            const double all_ms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            std::fprintf(stderr, "mt thread %d: jumps %.3f ms, total %.3f ms (%lld rows)\n", t, jump_ms, all_ms,
                         (long long)(ob - oa));
        }
    };
    std::vector<std::thread> pool;
    pool.reserve(T - 1);
    for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    if (last_end[T - 1] == n_rows) {
        g = gs[T - 1];                                     // it drew the stream's last word
    } else {                                               // NumPy's representation: the block of the last word
        const int64_t p = g.pos + 2 * n_rows * A;
        const int64_t q = (p + kN - 1) / kN - 1;
        Mt19937 fin;
        if (q == 0) fin = g;
        else mt_jump_blocks(g, q, fin);
        fin.pos = (int32_t)(p - q * kN);
        g = fin;
    }
    if (chunk_rc) {
        *chunk_rc = 0;
        for (int t = 0; t < T; ++t)
            if (rcs[t]) { *chunk_rc = rcs[t]; break; }
    }
    return T;
}

}  // namespace bcmpc
