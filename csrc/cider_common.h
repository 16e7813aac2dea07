// CIDEr-D shared definitions (host + device).
//
// An n-gram (n <= 4) of token ids is packed exactly into 64 bits: token t of
// position i occupies bits [16i, 16i+16) as t + 1, so 0 is "unused" and the
// key is collision-free for vocabularies up to 65534 ids (same packing as
// cst_captioning_amd/prepro/ciderdf.py:pack_ngram).
//
// The document-frequency table is an open-addressing hash table with linear
// probing: keys[cap] (0 = empty), vals[cap], cap a power of two.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define CST_HD __host__ __device__ __forceinline__
#else
#define CST_HD inline
#endif

namespace cst {

CST_HD uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

CST_HD int ngram_order(uint64_t key) {
  return 1 + ((key >> 16) != 0) + ((key >> 32) != 0) + ((key >> 48) != 0);
}

// df lookup; 0 when absent (the upstream scorer's defaultdict(float))
CST_HD float df_lookup(const int64_t* keys, const float* vals, uint32_t cap, uint64_t key) {
  uint32_t h = (uint32_t)mix64(key) & (cap - 1);
  for (uint32_t probe = 0; probe < cap; ++probe) {
    uint64_t k = (uint64_t)keys[h];
    if (k == key) return vals[h];
    if (k == 0) return 0.f;
    h = (h + 1) & (cap - 1);
  }
  return 0.f;
}

}  // namespace cst
