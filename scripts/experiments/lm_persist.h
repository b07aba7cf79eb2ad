// lm_persist.h — the persistent one-row decode step (lm_persist.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lm_kernels.h"

namespace tts {

struct PersistArgs {
  static constexpr int kMaxLayers = 32;
  const bf16_t* w[kMaxLayers][4] = {};   // tiled qkv, o, gate/up, down of each layer
  const bf16_t* ln[kMaxLayers][2] = {};  // ln1, ln2
  int L = 0;
  bf16_t* x = nullptr;                  // residual row: layer-0 input, last layer's output
  const int* row_slot = nullptr;        // [1] KV slot of the row
  const int* row_pos = nullptr;         // [1] position of the row's token
  bf16_t* kv = nullptr;                 // KV cache [L][K|V][slots][KVH][max_seq][D]
  long long kv_layer = 0;               // elements of one layer's K (or V) cache
  int max_seq = 0;
  const bf16_t* rope_cos = nullptr;     // [max_seq][D]
  const bf16_t* rope_sin = nullptr;
  float scale = 0.f, eps = 0.f;
  int NS = 0;                           // decode attention chunks per row (nsplit_decode)
  uint64_t* gran = nullptr;             // [L][slab] granules (memset 0xff)
  int* flags = nullptr;                 // [L][slab] producer flags (memset 0)
  int* err = nullptr;                   // set when a wait timed out
  int* seq = nullptr;                   // the step's tag (>= 1), advanced by the launch
  int ur_qkv = 0, ur_o = 0, ur_gu = 0, ur_d = 0;  // units per round of each matrix's layout
  unsigned long long* trace = nullptr;  // diagnostics: [256][L][32] phase timestamps (100 MHz) or null
};

size_t persist_gran_elems(int L);
size_t persist_flag_elems(int L);
// geometry check (TTS-1 dims, 256 CUs, decode chunks of 128, <= 8 chunks); fills ur[4]
bool persist_supported(int hidden, int heads, int kv_heads, int head_dim, int ffn, int L, int max_seq, int nsplit,
                       int split, int num_cu, int* ur);
void persist_init();  // kernel attributes (once, outside graph capture)
void launch_persist_step(const PersistArgs& a, hipStream_t s);

}  // namespace tts
