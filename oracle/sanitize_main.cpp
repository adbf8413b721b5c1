// ============================================================================
// TEST INFRASTRUCTURE ONLY — sanitizer driver for the CPU parity oracle
// (SURVEY.md §5 "Race detection": ASan/UBSan on the CPU restatement).
//
// Built by `make -C oracle sanitize` together with ctc_oracle.cpp under
// -fsanitize=address,undefined (no GPU code involved) and run by
// tests/test_oracle.py::test_oracle_under_sanitizers.  It drives every entry
// point of the oracle over the edge cases the parity tests use — T = 1,
// beam wider than the state space, ties (uniform emissions), zero
// probabilities, log input, a blank that is not label 0 with codes that flip
// the fold order, truncated outputs, bad arguments, several threads — and
// checks a few invariants of the results; any sanitizer report aborts with a
// non-zero status.
// ============================================================================
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

extern "C" {
int oracle_ctc_decode(const float*, int, int, int, int, int, const int32_t*, int, int, int, int,
                      int32_t*, int32_t*, int32_t*, double*);
int oracle_ctc_decode_prob(const float*, int, int, int, int, int, const int32_t*, int, int, int,
                           int, int32_t*, int32_t*, int32_t*, double*);
double oracle_ctc_time(const float*, int, int, int, int, int, int, int);
int oracle_ctc_decode_ts(const float*, int, int, int, int, int, const int32_t*, int, int, int, int,
                         int32_t*, int32_t*, int32_t*, double*, int32_t*);
}

namespace {

int failures = 0;

void expect(bool ok, const char* what, int T, int V, int beam) {
    if (!ok) {
        std::fprintf(stderr, "FAIL %s (T=%d V=%d beam=%d)\n", what, T, V, beam);
        failures++;
    }
}

// softmax of N(0, sigma^2) logits per frame, mt19937_64 seeded per case
std::vector<float> emissions(int T, int B, int V, uint64_t seed, double sigma, bool log_out) {
    std::mt19937_64 g(seed);
    std::normal_distribution<double> n(0.0, sigma);
    std::vector<float> e((size_t)T * B * V);
    std::vector<double> z(V);
    for (int t = 0; t < T; t++)
        for (int b = 0; b < B; b++) {
            double mx = -INFINITY, s = 0.0;
            for (int v = 0; v < V; v++) { z[v] = n(g); mx = std::max(mx, z[v]); }
            for (int v = 0; v < V; v++) s += std::exp(z[v] - mx);
            for (int v = 0; v < V; v++)
                e[((size_t)t * B + b) * V + v] =
                    (float)(log_out ? (z[v] - mx) - std::log(s) : std::exp(z[v] - mx) / s);
        }
    return e;
}

void run(const std::vector<float>& e, int T, int B, int V, int beam, int blank, const int32_t* codes,
         int is_log, int threads, int max_hyps, int max_len, bool prob) {
    std::vector<int32_t> nh(B), len((size_t)B * max_hyps), lab((size_t)B * max_hyps * max_len);
    std::vector<double> lp((size_t)B * max_hyps);
    const int rc = (prob ? oracle_ctc_decode_prob : oracle_ctc_decode)(
        e.data(), T, B, V, beam, blank, codes, is_log, threads, max_hyps, max_len, nh.data(),
        len.data(), lab.data(), lp.data());
    expect(rc == 0, "rc", T, V, beam);
    for (int b = 0; b < B; b++) {
        expect(nh[b] >= 1, "at least one hypothesis", T, V, beam);
        const int n = std::min<int>(nh[b], max_hyps);
        for (int k = 0; k < n; k++) {
            const size_t base = (size_t)b * max_hyps + k;
            expect(len[base] >= 0 && len[base] <= T, "length in [0, T]", T, V, beam);
            if (k > 0) expect(lp[base] <= lp[base - 1], "ranked by score", T, V, beam);
            for (int i = 0; i < std::min<int>(len[base], max_len); i++) {
                const int l = lab[base * max_len + i];
                expect(l >= 0 && l < V && l != blank, "label range, no blank", T, V, beam);
            }
        }
    }
}

}  // namespace

int main() {
    // ordinary shapes, single and multi-threaded, both score domains
    for (int prob = 0; prob < 2; prob++) {
        run(emissions(1, 3, 5, 1, 3.0, false), 1, 3, 5, 3, 0, nullptr, 0, 1, 8, 1, prob);
        run(emissions(12, 4, 6, 2, 3.0, false), 12, 4, 6, 4, 0, nullptr, 0, 3, 16, 12, prob);
        run(emissions(30, 5, 29, 3, 3.0, false), 30, 5, 29, 10, 0, nullptr, 0, 4, 32, 30, prob);
    }
    // beam wider than the state space (F2: nothing pruned)
    run(emissions(4, 2, 3, 4, 1.0, false), 4, 2, 3, 100, 0, nullptr, 0, 2, 256, 4, false);
    // uniform emissions: many exact ties at the cutoff, truncated outputs
    {
        const int T = 6, B = 2, V = 4;
        std::vector<float> u((size_t)T * B * V, 0.25f);
        run(u, T, B, V, 3, 0, nullptr, 0, 2, 5, 3, false);
    }
    // zero probabilities (log(0) = -inf scores)
    {
        std::vector<float> z = emissions(10, 2, 7, 5, 3.0, false);
        for (int v = 0; v < 7; v++) z[v] = v == 3 ? 1.0f : 0.0f;
        run(z, 10, 2, 7, 5, 0, nullptr, 0, 1, 16, 10, false);
    }
    // log input; blank = V-1 with a blank code above every symbol
    run(emissions(20, 3, 9, 6, 3.0, true), 20, 3, 9, 7, 0, nullptr, 1, 2, 16, 20, false);
    {
        std::vector<int32_t> codes(9);
        for (int v = 0; v < 8; v++) codes[v] = 'a' + v;
        codes[8] = '~';
        run(emissions(20, 3, 9, 7, 3.0, false), 20, 3, 9, 7, 8, codes.data(), 0, 2, 16, 20, false);
    }
    // large vocabulary, wide beam (C5-like, short T)
    run(emissions(5, 2, 300, 8, 3.0, false), 5, 2, 300, 40, 0, nullptr, 0, 2, 64, 5, false);
    // timesteps (ctcdecode's output): one strictly increasing frame < T per label
    {
        const int T = 25, B = 3, V = 11, beam = 6, mh = 16;
        std::vector<float> e = emissions(T, B, V, 10, 3.0, false);
        std::vector<int32_t> nh(B), len((size_t)B * mh), lab((size_t)B * mh * T), ts((size_t)B * mh * T);
        std::vector<double> lp((size_t)B * mh);
        expect(oracle_ctc_decode_ts(e.data(), T, B, V, beam, 0, nullptr, 0, 2, mh, T, nh.data(), len.data(),
                                    lab.data(), lp.data(), ts.data()) == 0, "ts rc", T, V, beam);
        for (int b = 0; b < B; b++)
            for (int k = 0; k < std::min(nh[b], mh); k++) {
                const size_t base = (size_t)b * mh + k;
                for (int i = 0; i < len[base]; i++) {
                    const int f = ts[base * T + i];
                    expect(f >= 0 && f < T && (i == 0 || f > ts[base * T + i - 1]), "timesteps increasing",
                           T, V, beam);
                }
            }
    }
    // timing entry point
    {
        std::vector<float> e = emissions(8, 2, 29, 9, 3.0, false);
        expect(oracle_ctc_time(e.data(), 8, 2, 29, 5, 0, 0, 2) >= 0.0, "time", 8, 29, 5);
    }
    // bad arguments are rejected, not read
    {
        int32_t nh = 0, len = 0, lab = 0;
        double lp = 0.0;
        float e = 1.0f;
        expect(oracle_ctc_decode(&e, 1, 1, 1, 1, 0, nullptr, 0, 1, 1, 1, &nh, &len, &lab, &lp) != 0,
               "V=1 rejected", 1, 1, 1);
        expect(oracle_ctc_decode(&e, 0, 1, 2, 1, 0, nullptr, 0, 1, 1, 1, &nh, &len, &lab, &lp) != 0,
               "T=0 rejected", 0, 2, 1);
    }
    if (failures) return 1;
    std::printf("oracle sanitizer run: ok\n");
    return 0;
}
