// Host-side stress driver for csrc/host/cider_host.cpp (the CIDEr-D table
// builder and CPU scorer), built with AddressSanitizer + UBSan by
// tests/test_native_sanitizers.py.  Exercises random datasets plus edge cases
// (empty / EOS-only / BOS-only captions, videos without references, maximal
// lengths, use_eos on and off) and checks basic invariants of the scores.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "host/cider_host.h"

using namespace cst;

static uint64_t pack(const std::vector<int>& t, int i, int n) {
  uint64_t k = 0;
  for (int j = 0; j < n; ++j) k |= (uint64_t)(t[i + j] + 1) << (16 * j);
  return k;
}

static int run(uint32_t seed, int Nv, int L, int V, int use_eos) {
  std::mt19937 rng(seed);
  std::vector<int64_t> start(Nv), end(Nv), labels;
  int M = 0;
  for (int v = 0; v < Nv; ++v) {
    const int ncap = (v % 7 == 3) ? 0 : 1 + (int)(rng() % 24);  // some videos have no refs
    start[v] = M;
    for (int c = 0; c < ncap; ++c, ++M) {
      const int len = (int)(rng() % (L + 1));
      const int kind = (int)(rng() % 16);
      for (int i = 0; i < L; ++i) {
        int64_t tok = i < len ? 2 + (int64_t)(rng() % (V - 2)) : 0;
        if (kind == 0) tok = 0;                 // empty caption
        if (kind == 1 && i == 0) tok = 1;       // leading BOS (skipped)
        labels.push_back(tok);
      }
    }
    end[v] = M;  // exclusive
  }
  // df over the reference n-grams (plus unrelated keys)
  std::vector<int64_t> df_keys;
  std::vector<float> df_vals;
  for (int m = 0; m < M; ++m) {
    std::vector<int> toks;
    for (int i = 0; i < L; ++i) {
      const int t = (int)labels[(size_t)m * L + i];
      if (t == 0) {
        if (use_eos) toks.push_back(0);
        break;
      }
      if (t != 1) toks.push_back(t);
    }
    for (int n = 1; n <= 4; ++n)
      for (int i = 0; i + n <= (int)toks.size(); ++i) {
        df_keys.push_back((int64_t)pack(toks, i, n));
        df_vals.push_back(1.f + (float)(rng() % 5));
      }
  }
  for (int i = 0; i < 100; ++i) {
    df_keys.push_back((int64_t)(rng() | 1));
    df_vals.push_back(3.f);
  }
  const double log_ref_len = std::log((double)std::max(Nv, 2));
  CiderTables t = build_cider_tables(labels.data(), M, L, start.data(), end.data(), Nv,
                                     df_keys.data(), df_vals.data(), (int)df_keys.size(),
                                     log_ref_len, use_eos);
  CiderTablesView view{t.ht_cap, t.ht_keys.data(), t.ht_vals.data(), t.vid_ref_off.data(),
                       t.ref_ng_off.data(), t.ref_norm.data(), t.ref_len.data(),
                       t.ng_key.data(), t.ng_val.data()};
  // hypotheses: random, copies of references, all-EOS, full length
  const int T = std::min(L, 63), N = 3 * Nv;
  std::vector<int64_t> hyps((size_t)N * T, 0), hv(N);
  for (int i = 0; i < N; ++i) {
    const int v = i % Nv;
    hv[i] = v;
    const int kind = i % 3;
    for (int j = 0; j < T; ++j) {
      if (kind == 0) hyps[(size_t)i * T + j] = 2 + (int64_t)(rng() % (V - 2));
      if (kind == 1 && end[v] > start[v]) hyps[(size_t)i * T + j] = labels[(size_t)start[v] * L + j];
    }
  }
  std::vector<float> out(N, -1.f);
  cider_score_host(hyps.data(), N, T, hv.data(), view, log_ref_len, use_eos, out.data());
  for (int i = 0; i < N; ++i) {
    if (!std::isfinite(out[i]) || out[i] < 0.f) {
      std::printf("bad score %d: %f\n", i, out[i]);
      return 1;
    }
  }
  return 0;
}

int main() {
  int bad = 0;
  for (uint32_t s = 0; s < 6; ++s)
    for (int use_eos = 0; use_eos < 2; ++use_eos) {
      bad |= run(s, 40 + 13 * (int)s, 30, 300 + 97 * (int)s, use_eos);
      bad |= run(100 + s, 5, 63, 12, use_eos);  // tiny vocab: many repeated n-grams
    }
  std::printf(bad ? "FAILED\n" : "ok\n");
  return bad;
}
