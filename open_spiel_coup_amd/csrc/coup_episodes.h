// coup_episodes.h -- the per-lane episode accumulators of the step,
// trajectory and rollout kernels (2-player coup_kernels.hip and N-player
// coup_nplayer.hip): per lane, the episodes that ended and the sum of player
// 0's Returns() over them (coup.cc:1016-1032), the quantity the multi-GPU
// job all-gathers.
//
// Two forms, chosen by the caller (coup_step_outputs / coup_rollout_stats):
//  - pair: int32 episodes[B] and return_sum[B] -- 8 bytes per lane each way;
//  - packed: ONE word per lane, return_sum << S | episodes (two's complement,
//    S = 8 for an int16 word, 16 for an int32 word).  The word is the
//    collective's payload as it stands, so no packing kernel runs between the
//    steps and the all-gather, and an int16 word moves 2 bytes per lane each
//    way instead of 8.  The fields do not saturate: the caller bounds the
//    steps between clears (int16: episodes <= 255 and |return_sum| <= 127,
//    i.e. 2(N-1) K <= 127; bench.py payload_width, BatchedCoupEnv's fold).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "coup_mi355x.h"

namespace coup {

// A lane's accumulator value as two scalars.  Not an int2: HIP's int2 is a
// <2 x i32> IR vector, and <2 x i32> values carried through the rules'
// divergent control flow are the shape the AMDGPU backend lowers wrong
// (DESIGN.md section 12); a struct of two ints is split into two scalars.
struct EpVal {
  int32_t x, y;
};

struct EpAcc {
  int32_t* count;      // pair form
  int32_t* ret;
  void* word;          // packed form (count == ret == nullptr)
  int32_t word_bytes;  // 2 or 4 with `word`

  __device__ __forceinline__ bool on() const { return count != nullptr || word != nullptr; }

  // The lane's current value: (episodes, return sum), or (word, 0) packed.
  __device__ __forceinline__ EpVal load(int64_t i) const {
    if (word)
      return EpVal{word_bytes == 2 ? (int32_t) static_cast<const int16_t*>(word)[i]
                                   : static_cast<const int32_t*>(word)[i],
                   0};
    if (count) return EpVal{count[i], ret[i]};
    return EpVal{0, 0};
  }

  // Store `prev` (a load()) plus `eps` episodes whose returns sum to `r`.
  // Unsigned arithmetic: the packed word is (return_sum * 2^S + episodes)
  // modulo 2^(8 * word_bytes).
  __device__ __forceinline__ void store(int64_t i, EpVal prev, int32_t eps, int32_t r) const {
    if (word) {
      const uint32_t w = (uint32_t)prev.x + ((uint32_t)r << (4 * word_bytes)) + (uint32_t)eps;
      if (word_bytes == 2)
        static_cast<int16_t*>(word)[i] = (int16_t)w;
      else
        static_cast<int32_t*>(word)[i] = (int32_t)w;
    } else if (count) {
      count[i] = prev.x + eps;
      ret[i] = prev.y + r;
    }
  }

  // Load, add, store (the fused kernels, once per launch).
  __device__ __forceinline__ void add(int64_t i, int32_t eps, int32_t r) const {
    if (on()) store(i, load(i), eps, r);
  }
};

// Host: the accumulators a call's outputs name (out / stats may be null:
// none).  Returns nullptr, or what is malformed.
template <class Out>
inline const char* ep_acc_of(const Out* out, EpAcc& e) {
  e = EpAcc{nullptr, nullptr, nullptr, 0};
  if (!out) return nullptr;
  if ((out->episodes == nullptr) != (out->return_sum == nullptr)) return "episodes and return_sum go together";
  if (out->episode_word && out->episodes) return "episode_word replaces episodes / return_sum: not both";
  if (out->episode_word && out->episode_word_bytes != 2 && out->episode_word_bytes != 4)
    return "episode_word_bytes must be 2 or 4";
  e.count = out->episodes;
  e.ret = out->return_sum;
  e.word = out->episode_word;
  e.word_bytes = out->episode_word ? out->episode_word_bytes : 0;
  return nullptr;
}

}  // namespace coup
