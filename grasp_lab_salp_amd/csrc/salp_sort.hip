// salp_sort.hip — launch order of the lock-step kernels (salp_step,
// salp_step_random): envs sorted by the predicted length of the breathing
// cycle each will run, longest first.
//
// A lock-step launch ends when its slowest wave ends, and a wave when its
// slowest lane ends (cycle lengths under random actions: mean 710 ticks, wave64
// max/mean ~1.8, SURVEY.md §7 hard part 1).  While every wave is resident at
// once (n_envs <= one wave per SIMD) nothing can shorten the launch: it lasts
// the longest cycle of the batch.  Beyond that, waves run in rounds per SIMD;
// sorting makes the lanes of a wave similar (little idle) and hands the long
// waves out first, so the rounds pack.  Per-env results do not depend on the
// order (envs are independent): parity holds by construction and is tested.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>

// Temporary storage bytes for sorting n (uint32 key, int32 id) pairs.
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_sort_temp_bytes(int64_t n, size_t* bytes) {
    *bytes = 0;
    return hipcub::DeviceRadixSort::SortPairsDescending(nullptr, *bytes, (const uint32_t*)nullptr,
                                                        (uint32_t*)nullptr, (const int32_t*)nullptr,
                                                        (int32_t*)nullptr, (int)n, 0, 16, (hipStream_t)nullptr);
}

// keys (predicted ticks, < 2^16) descending, carrying the env ids into `order`.
extern "C" __attribute__((visibility("hidden"))) hipError_t salp_sort_launch(
    void* temp, size_t temp_bytes, const uint32_t* keys_in, uint32_t* keys_out, const int32_t* ids_in,
    int32_t* order, int64_t n, void* stream) {
    size_t bytes = temp_bytes;
    return hipcub::DeviceRadixSort::SortPairsDescending(temp, bytes, keys_in, keys_out, ids_in, order, (int)n, 0, 16,
                                                        (hipStream_t)stream);
}
