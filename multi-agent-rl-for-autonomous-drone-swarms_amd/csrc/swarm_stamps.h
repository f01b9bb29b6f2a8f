// swarm_stamps.h — diagnostic phase timestamps of the step kernels (tools/stamps.py,
// tools/stamps16.py).  Only the stamps build (`python tools/stamps.py build`: one translation unit,
// -DSWARM_STAMPS) defines SWARM_STAMPS; in the product build every macro below is empty.
//
// Record layout, one 16-word record per env (first 65,536 envs): words 0-8 the s_memtime of
// phase boundaries 0..8, 9 HW_ID, 10 XCC_ID, 11 / 12 s_memrealtime at the wave's start / end,
// 13 step16q's slow-path flags.
#pragma once

#ifdef SWARM_STAMPS
__device__ unsigned long long g_stamps[1 << 20];
// phase boundary i of record `rec` (lane 0 of the wave writes)
#define STAMP_AT(rec, i)                                                                 \
  do {                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    unsigned long long ts_;                                                              \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts_)::"memory");           \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    if ((threadIdx.x & 63) == 0 && (rec) < (1 << 16)) g_stamps[(rec) * 16 + (i)] = ts_;  \
  } while (0)
// the wave's realtime start, and its realtime end with the hardware placement (`lead`: the
// writing thread)
#define STAMP_BEGIN(rec, lead)                                                           \
  do {                                                                                   \
    if ((lead) && (rec) < (1 << 16)) g_stamps[(rec) * 16 + 11] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define STAMP_END(rec, lead)                                                             \
  do {                                                                                   \
    if ((lead) && (rec) < (1 << 16)) {                                                   \
      g_stamps[(rec) * 16 + 9] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);    \
      g_stamps[(rec) * 16 + 10] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);  \
      g_stamps[(rec) * 16 + 12] = __builtin_amdgcn_s_memrealtime();                      \
    }                                                                                    \
  } while (0)
// step16q: slow paths a wave took (1 / 16 quad exact selection, 2 exact collision band, 4 reset,
// 8 masked pass), OR-ed over the wave into word 13
#define Q16_FLAGS_DECL uint32_t q16_flags = 0u
#define Q16_FLAG(f) (q16_flags |= (f))
#define Q16_FLAGS_END(rec, lane)                                                         \
  do {                                                                                   \
    uint32_t fw_ = 0u;                                                                   \
    for (uint32_t bit_ = 1u; bit_ <= 16u; bit_ <<= 1)                                    \
      fw_ |= __ballot((q16_flags & bit_) != 0u) != 0 ? bit_ : 0u;                        \
    if ((lane) == 0 && (rec) < (1 << 16)) g_stamps[(rec) * 16 + 13] = fw_;               \
  } while (0)
#define STAMP_VAR(decl) decl
#else
#define STAMP_AT(rec, i) do {} while (0)
#define STAMP_BEGIN(rec, lead) do {} while (0)
#define STAMP_END(rec, lead) do {} while (0)
#define Q16_FLAGS_DECL do {} while (0)
#define Q16_FLAG(f) ((void)0)
#define Q16_FLAGS_END(rec, lane) do {} while (0)
#define STAMP_VAR(decl)
#endif
#define STAMP(i) STAMP_AT(blockIdx.x, i)
