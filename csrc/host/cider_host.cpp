// Native host side of CIDEr-D (no torch dependency).
//
//  * build_cider_tables: once per dataset, turns every GT label row into its
//    CIDEr-D reference vector (array_to_str semantics of
//    /root/reference/utils.py:135-152, tf-idf with the df table of
//    compute_ciderdf.py:56-70, per-order L2 norms, bigram-occurrence length)
//    and builds the open-addressing df hash table the GPU kernel probes.
//  * cider_score_host: the same scorer in double precision on the CPU (used
//    when no GPU is present and as a fast oracle in tests).
#include "cider_host.h"

#include <algorithm>
#include <cmath>
#include <unordered_map>

#include "../cider_common.h"

namespace cst {

static void compact_tokens(const int64_t* row, int T, int use_eos, std::vector<int>& out) {
  out.clear();
  for (int i = 0; i < T; ++i) {
    const int t = (int)row[i];
    if (t == 0) {
      if (use_eos) out.push_back(0);
      return;
    }
    if (t == 1) continue;
    out.push_back(t);
  }
}

static void count_ngrams(const std::vector<int>& toks, std::vector<std::pair<uint64_t, int>>& out) {
  std::unordered_map<uint64_t, int> cnt;
  const int W = (int)toks.size();
  for (int n = 1; n <= 4; ++n) {
    for (int i = 0; i + n <= W; ++i) {
      uint64_t key = 0;
      for (int j = 0; j < n; ++j) key |= (uint64_t)(toks[i + j] + 1) << (16 * j);
      cnt[key] += 1;
    }
  }
  out.assign(cnt.begin(), cnt.end());
  std::sort(out.begin(), out.end());
}

static uint32_t next_pow2(uint64_t x) {
  uint32_t c = 1;
  while (c < x) c <<= 1;
  return c;
}

CiderTables build_cider_tables(const int64_t* labels, int M, int L, const int64_t* start,
                               const int64_t* end, int Nv, const int64_t* df_keys,
                               const float* df_vals, int n_df, double log_ref_len,
                               int use_eos) {
  CiderTables t;
  t.ht_cap = next_pow2((uint64_t)std::max(16, 2 * n_df));
  t.ht_keys.assign(t.ht_cap, 0);
  t.ht_vals.assign(t.ht_cap, 0.f);
  for (int i = 0; i < n_df; ++i) {
    const uint64_t k = (uint64_t)df_keys[i];
    uint32_t h = (uint32_t)mix64(k) & (t.ht_cap - 1);
    while (t.ht_keys[h] != 0 && (uint64_t)t.ht_keys[h] != k) h = (h + 1) & (t.ht_cap - 1);
    t.ht_keys[h] = (int64_t)k;
    t.ht_vals[h] = df_vals[i];
  }
  t.vid_ref_off.resize(Nv + 1);
  t.ref_ng_off.push_back(0);
  std::vector<int> toks;
  std::vector<std::pair<uint64_t, int>> grams;
  int nref = 0;
  for (int v = 0; v < Nv; ++v) {
    t.vid_ref_off[v] = nref;
    for (int64_t r = start[v]; r < end[v]; ++r) {
      compact_tokens(labels + r * L, L, use_eos, toks);
      count_ngrams(toks, grams);
      double norm[4] = {0, 0, 0, 0};
      for (auto& g : grams) {
        const float df = df_lookup(t.ht_keys.data(), t.ht_vals.data(), t.ht_cap, g.first);
        const double val = (double)g.second * (log_ref_len - std::log(std::max(1.0, (double)df)));
        norm[ngram_order(g.first) - 1] += val * val;
        t.ng_key.push_back((int64_t)g.first);
        t.ng_val.push_back((float)val);
      }
      for (int n = 0; n < 4; ++n) t.ref_norm.push_back((float)std::sqrt(norm[n]));
      t.ref_len.push_back(std::max((int)toks.size() - 1, 0));
      t.ref_ng_off.push_back((int32_t)t.ng_key.size());
      ++nref;
    }
  }
  t.vid_ref_off[Nv] = nref;
  return t;
}

void cider_score_host(const int64_t* hyps, int N, int T, const int64_t* hyp_video,
                      const CiderTablesView& t, double log_ref_len, int use_eos,
                      float* out) {
  std::vector<int> toks;
  std::vector<std::pair<uint64_t, int>> grams;
  for (int i = 0; i < N; ++i) {
    compact_tokens(hyps + (int64_t)i * T, T, use_eos, toks);
    count_ngrams(toks, grams);
    std::unordered_map<uint64_t, double> vh;
    double nh[4] = {0, 0, 0, 0};
    for (auto& g : grams) {
      const float df = df_lookup(t.ht_keys, t.ht_vals, t.ht_cap, g.first);
      const double val = (double)g.second * (log_ref_len - std::log(std::max(1.0, (double)df)));
      vh[g.first] = val;
      nh[ngram_order(g.first) - 1] += val * val;
    }
    for (int n = 0; n < 4; ++n) nh[n] = std::sqrt(nh[n]);
    const double lh = std::max((int)toks.size() - 1, 0);
    const int v = (int)hyp_video[i];
    const int r0 = t.vid_ref_off[v], r1 = t.vid_ref_off[v + 1];
    double total = 0;
    for (int r = r0; r < r1; ++r) {
      double acc[4] = {0, 0, 0, 0};
      for (int g = t.ref_ng_off[r]; g < t.ref_ng_off[r + 1]; ++g) {
        auto it = vh.find((uint64_t)t.ng_key[g]);
        if (it == vh.end()) continue;
        const double vr = t.ng_val[g];
        acc[ngram_order((uint64_t)t.ng_key[g]) - 1] += std::min(it->second, vr) * vr;
      }
      const double delta = lh - t.ref_len[r];
      const double pen = std::exp(-(delta * delta) / 72.0);
      for (int n = 0; n < 4; ++n) {
        double val = acc[n];
        const double nr = t.ref_norm[r * 4 + n];
        if (nh[n] != 0 && nr != 0) val /= (nh[n] * nr);
        total += val * pen;
      }
    }
    out[i] = (r1 > r0) ? (float)(10.0 * total / (4.0 * (r1 - r0))) : 0.f;
  }
}

}  // namespace cst
