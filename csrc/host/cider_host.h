#pragma once
#include <stdint.h>

#include <vector>

namespace cst {

struct CiderTables {
  uint32_t ht_cap = 0;
  std::vector<int64_t> ht_keys;
  std::vector<float> ht_vals;
  std::vector<int32_t> vid_ref_off;
  std::vector<int32_t> ref_ng_off;
  std::vector<float> ref_norm;
  std::vector<int32_t> ref_len;
  std::vector<int64_t> ng_key;
  std::vector<float> ng_val;
};

struct CiderTablesView {
  uint32_t ht_cap;
  const int64_t* ht_keys;
  const float* ht_vals;
  const int32_t* vid_ref_off;
  const int32_t* ref_ng_off;
  const float* ref_norm;
  const int32_t* ref_len;
  const int64_t* ng_key;
  const float* ng_val;
};

CiderTables build_cider_tables(const int64_t* labels, int M, int L, const int64_t* start,
                               const int64_t* end, int Nv, const int64_t* df_keys,
                               const float* df_vals, int n_df, double log_ref_len, int use_eos);

void cider_score_host(const int64_t* hyps, int N, int T, const int64_t* hyp_video,
                      const CiderTablesView& t, double log_ref_len, int use_eos, float* out);

}  // namespace cst
