// Microbenchmark + stale-read stress test of the persistent kernels' per-tick hand-off, by
// transport form (the two-layer wavefront forward's shape: 8 columns x 32 workgroups, every
// workgroup reads both layers' 32 KB ring slots of its column per tick and each of its 4 waves
// publishes 512 B).
//
//   mode 0  sc1 payload stores, vmcnt(0), one atomic counter add per storing wave; sc1 poll
//           (what csrc/persist_common.h does today: MI355X_MICROARCH.md "Valid forms", row 3)
//   mode 1  plain payload stores (the line stays in the producer XCD's L2), atomic counters
//   mode 2  plain payload stores + a plain per-wave flag store (tick number); one wave polls the
//           column's 64 flags per layer with one sc1 dword load per lane (all L2-resident)
//   mode 3  sc1 payload + sc1 per-wave flags (mode 2's poll with today's write-through stores)
//
// Modes 1-2 keep handed-off lines in ONE XCD's L2, so they are used only for a column whose 32
// workgroups all read the same HW_REG_XCC_ID at kernel start (an in-kernel exchange); any other
// column falls back to mode 0.  Every dword a consumer loads is a tag (the producing tick) and is
// checked: `stale` counts mismatches.  `jitter` adds a per-(workgroup, tick) pseudo-random delay
// before the producer stores (uneven load).
//
// Build: hipcc --offload-arch=gfx950 -O3 scripts/micro/handoff_xcd.hip -o build/micro/handoff_xcd
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int NCOL = 8, NWG = 32;  // columns x workgroups per column (256 workgroups)
constexpr int SLOT = 32 * 1024;    // bytes of one layer's ring slot per column
constexpr unsigned kSc1 = 16;

struct Args {
  unsigned* ring;              // [layer 2][slot 2][col][SLOT bytes]
  unsigned* cnt;               // [col][T + 1][16] (dwords 0 / 1: layer 0 / 1)
  unsigned* flags;             // [col][layer][64] tick+1 of each producing wave
  unsigned long long* xmask;   // [col] per-XCC arrival bytes
  unsigned* out;               // [0] stale, [1] err, [2] local workgroups
  int T, jitter, spin_limit;
};

__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}

template <int MODE>
__global__ void __launch_bounds__(256, 1) tick_kernel(Args a) {
  __shared__ unsigned pad[24 * 1024];  // 96 KB: one workgroup per CU
  __shared__ int loc_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x % NCOL, ubk = blockIdx.x / NCOL;
  const int T = a.T;
  if (threadIdx.x == 0) {
    pad[0] = 0;
    const unsigned x = xcc_id();
    __hip_atomic_fetch_add(&a.xmask[col], 1ull << (8 * x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long m = 0;
    int spins = 0;
    for (;;) {
      m = __hip_atomic_load(&a.xmask[col], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned s = 0;
      for (int i = 0; i < 8; ++i) s += (unsigned)(m >> (8 * i)) & 0xFFu;
      if (s >= NWG || ++spins > a.spin_limit) break;
      __builtin_amdgcn_s_sleep(1);
    }
    int l = 0;
    for (int i = 0; i < 8; ++i) l |= ((m >> (8 * i)) & 0xFFu) == NWG;
    loc_s = l;
    if (l) atomicAdd(&a.out[2], 1u);
  }
  __syncthreads();
  const bool loc = MODE != 0 && MODE != 3 && loc_s;  // modes 1/2 only on single-XCD columns
  const bool flagm = (MODE == 2 && loc) || MODE == 3;
  unsigned* cnt = a.cnt + (size_t)col * (T + 1) * 16;
  unsigned* fl = a.flags + (size_t)col * 2 * 64;
  unsigned stale = 0;
  bool dead = false;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      a.ring, (short)0, 2 * 2 * NCOL * SLOT, 0x00020000);
  for (int tau = 0; tau < T; ++tau) {
    if (tau >= 1 && !dead) {
      if (flagm) {
        if (w == 0) {
          int spins = 0;
          for (;;) {
            const unsigned f0 = __hip_atomic_load(fl + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned f1 = __hip_atomic_load(fl + 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__all(f0 >= (unsigned)tau && f1 >= (unsigned)tau)) break;
            if (++spins > a.spin_limit) {
              dead = true;
              if (lane == 0) atomicAdd(&a.out[1], 1u);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
      } else if (threadIdx.x == 0) {
        int spins = 0;
        for (;;) {
          const unsigned c0 = __hip_atomic_load(cnt + tau * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const unsigned c1 = __hip_atomic_load(cnt + tau * 16 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (c0 >= 64 && c1 >= 64) break;
          if (++spins > a.spin_limit) {
            dead = true;
            atomicAdd(&a.out[1], 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    __syncthreads();
    if (tau >= 1) {
      // this wave's quarter of both layers' slots: 2 x 8 KB = 16 loads of 16 B per lane
      u32x4 v[16];
#pragma unroll
      for (int l = 0; l < 2; ++l)
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const unsigned off = (unsigned)(((l * 2 + (tau & 1)) * NCOL + col) * SLOT +
                                          w * 8192 + (s * 64 + lane) * 16);
          v[l * 8 + s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, kSc1));
        }
#pragma unroll
      for (int i = 0; i < 16; ++i)
        stale += (v[i][0] != (unsigned)tau) + (v[i][1] != (unsigned)tau) +
                 (v[i][2] != (unsigned)tau) + (v[i][3] != (unsigned)tau);
    }
    __syncthreads();
    if (a.jitter) {
      const unsigned h = (blockIdx.x * 2654435761u) ^ (tau * 40503u);
      const int n = (int)((h >> 13) & 3u) * a.jitter;
      for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(8);
    }
    if (tau + 1 < T) {
      const int L = w >> 1, J = w & 1;
      const unsigned tag = (unsigned)(tau + 1);
      const size_t off = ((size_t)((L * 2 + ((tau + 1) & 1)) * NCOL + col) * SLOT +
                          ((ubk * 2 + J) * 64 + lane) * 8) / 4;
      const unsigned long long v2 = ((unsigned long long)tag << 32) | tag;
      if (loc && MODE != 3)
        *reinterpret_cast<unsigned long long*>(a.ring + off) = v2;
      else
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.ring + off), v2, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        if (flagm) {
          if (MODE == 3)
            __hip_atomic_store(fl + L * 64 + ubk * 2 + J, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else
            __hip_atomic_store(fl + L * 64 + ubk * 2 + J, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // sc0: as the kernels
        } else {
          __hip_atomic_fetch_add(cnt + (tau + 1) * 16 + L, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
  if (stale) atomicAdd(&a.out[0], stale);
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 2000;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  Args a{};
  a.T = T;
  a.spin_limit = 1 << 22;
  hipMalloc(&a.ring, 2 * 2 * NCOL * SLOT);
  hipMalloc(&a.cnt, sizeof(unsigned) * NCOL * (T + 1) * 16);
  hipMalloc(&a.flags, sizeof(unsigned) * NCOL * 2 * 64);
  hipMalloc(&a.xmask, sizeof(unsigned long long) * NCOL);
  hipMalloc(&a.out, 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const void* fns[4] = {(const void*)tick_kernel<0>, (const void*)tick_kernel<1>,
                        (const void*)tick_kernel<2>, (const void*)tick_kernel<3>};
  int bad = 0;
  for (int jit = 0; jit <= 4; jit += 4)
    for (int mode = 0; mode < 4; ++mode) {
      a.jitter = jit;
      float best = 1e30f;
      unsigned tot_stale = 0, tot_err = 0, locs = 0;
      for (int r = 0; r < reps; ++r) {
        hipMemset(a.ring, 0, 2 * 2 * NCOL * SLOT);
        hipMemset(a.cnt, 0, sizeof(unsigned) * NCOL * (T + 1) * 16);
        hipMemset(a.flags, 0, sizeof(unsigned) * NCOL * 2 * 64);
        hipMemset(a.xmask, 0, sizeof(unsigned long long) * NCOL);
        hipMemset(a.out, 0, 16);
        void* args[] = {&a};
        hipEventRecord(e0);
        hipLaunchKernel(fns[mode], dim3(NCOL * NWG), dim3(256), args, 0, 0);
        hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) { printf("sync failed\n"); return 2; }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
        unsigned o[3];
        hipMemcpy(o, a.out, 12, hipMemcpyDeviceToHost);
        tot_stale += o[0];
        tot_err += o[1];
        locs = o[2];
      }
      printf("mode %d jitter %d: %.3f us/tick  stale %u  timeouts %u  local workgroups %u/256  (%d x %d ticks)\n",
             mode, jit, best * 1e3f / T, tot_stale, tot_err, locs, reps, T);
      bad |= tot_stale != 0 || tot_err != 0;
    }
  return bad;
}
