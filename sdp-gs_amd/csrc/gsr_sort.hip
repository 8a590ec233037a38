// gsr_sort.hip -- device-wide prefix sum and stable LSD radix sort for gfx950 (wave64).
//
// Replaces the reference's CUB calls (cub::DeviceScan::InclusiveSum at
// cuda_rasterizer/rasterizer_impl.cu:277 and cub::DeviceRadixSort::SortPairs at :303-308, CUDA
// toolkit 11.6 per environment.yml:6).  The sort must be STABLE: the reference breaks equal-depth
// ties by emission order, i.e. by Gaussian index.
//
// Design: the prefix sum is reduce-then-scan (3 launches, no inter-workgroup hand-off); the radix
// sort is one-sweep (one launch per 8-bit pass with a decoupled look-back over agent-scope status
// words, see below), whose in-workgroup ranking uses wave64 ballots ("match" of the digit)
// instead of shared-memory per-thread counters.
#include <atomic>

#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
constexpr int kScanItems = kScanTile / kThreads;   // 8

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Inclusive wave64 scan.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Exclusive scan across a workgroup of NW waves; lds must hold NW u32.  Returns the exclusive
// prefix of v and the workgroup total.  Contains two __syncthreads().
template <int NW>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
  const int lane = lane_id();
  const int wid = (int)(threadIdx.x >> 6);
  uint32_t incl = wave_incl_scan(v);
  if (lane == 63) lds[wid] = incl;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    uint32_t c = lds[w];
    pre += (w < wid) ? c : 0u;
    tot += c;
  }
  __syncthreads();
  total = tot;
  return pre + incl - v;
}

template <bool GATHER>
__device__ __forceinline__ void scan_reduce_body(const uint32_t* __restrict__ in,
                                                 const uint32_t* __restrict__ gather, size_t n,
                                                 uint32_t* __restrict__ parts, uint32_t blk) {
  __shared__ uint32_t lds[kThreads / 64];
  const size_t base = (size_t)blk * kScanTile;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    size_t i = base + (size_t)k * kThreads + threadIdx.x;
    if (i < n) s += GATHER ? in[min(gather[i], (uint32_t)n - 1u)] : in[i];
  }
  uint32_t total;
  block_excl_scan<kThreads / 64>(s, lds, total);
  if (threadIdx.x == 0) parts[blk] = total;
}

template <bool GATHER>
__global__ __launch_bounds__(kThreads) void scan_reduce_kernel(const uint32_t* __restrict__ in,
                                                               const uint32_t* __restrict__ gather,
                                                               size_t n,
                                                               uint32_t* __restrict__ parts) {
  scan_reduce_body<GATHER>(in, gather, n, parts, blockIdx.x);
}

// One workgroup of 1024 threads: exclusive scan of the partials in place (<= kScanMaxParts).
__device__ __forceinline__ void scan_parts_body(uint32_t* __restrict__ parts, int n) {
  __shared__ uint32_t lds[16];
  constexpr int kPer = kScanMaxParts / 1024;
  uint32_t v[kPer];
  uint32_t s = 0;
  const int base = (int)threadIdx.x * kPer;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    v[k] = (base + k < n) ? parts[base + k] : 0u;
    s += v[k];
  }
  uint32_t total;
  uint32_t pre = block_excl_scan<16>(s, lds, total);
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    if (base + k < n) parts[base + k] = pre;
    pre += v[k];
  }
}

__global__ __launch_bounds__(1024) void scan_parts_kernel(uint32_t* __restrict__ parts, int n) {
  scan_parts_body(parts, n);
}

// A lane's kScanItems consecutive counts as 16-byte loads and stores when the arrays are aligned
// (workgroup-uniform test); else one 4-byte access per item.  RAW: parts holds the workgroups'
// plain sums (no scan_parts launch) and each workgroup adds up its predecessors' itself -- integer
// sums, so the same result; one launch fewer in the binning chain.
template <bool GATHER, bool INCLUSIVE, bool RAW = false>
__device__ __forceinline__ void scan_final_body(const uint32_t* __restrict__ in,
                                                const uint32_t* __restrict__ gather, size_t n,
                                                const uint32_t* __restrict__ parts,
                                                uint32_t* __restrict__ out, uint32_t blk) {
  static_assert(kScanItems % 4 == 0, "vector scan items");
  __shared__ uint32_t lds[kThreads / 64];
  const size_t base = (size_t)blk * kScanTile + (size_t)threadIdx.x * kScanItems;
  const bool vec = !GATHER && base + kScanItems <= n &&
                   (((uintptr_t)in | (uintptr_t)out) & 15u) == 0;
  uint32_t v[kScanItems];
  uint32_t s = 0;
  if (vec) {
#pragma unroll
    for (int k = 0; k < kScanItems; k += 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(in + base + k);
      v[k] = q.x;
      v[k + 1] = q.y;
      v[k + 2] = q.z;
      v[k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
      size_t i = base + k;
      v[k] = (i < n) ? (GATHER ? in[min(gather[i], (uint32_t)n - 1u)] : in[i]) : 0u;
    }
  }
#pragma unroll
  for (int k = 0; k < kScanItems; k++) s += v[k];
  uint32_t base_pre;
  if (RAW) {
    __shared__ uint32_t lds_p[kThreads / 64];
    uint32_t ps = 0;
    for (uint32_t q = threadIdx.x; q < blk; q += kThreads) ps += parts[q];
    block_excl_scan<kThreads / 64>(ps, lds_p, base_pre);  // base_pre = the workgroup's total
  } else {
    base_pre = parts[blk];
  }
  uint32_t total;
  uint32_t pre = block_excl_scan<kThreads / 64>(s, lds, total) + base_pre;
  uint32_t o[kScanItems];
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    uint32_t incl = pre + v[k];
    o[k] = INCLUSIVE ? incl : pre;
    pre = incl;
  }
  if (vec) {
#pragma unroll
    for (int k = 0; k < kScanItems; k += 4)
      *reinterpret_cast<uint4*>(out + base + k) = make_uint4(o[k], o[k + 1], o[k + 2], o[k + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < kScanItems; k++)
      if (base + k < n) out[base + k] = o[k];
  }
}

template <bool GATHER, bool INCLUSIVE>
__global__ __launch_bounds__(kThreads) void scan_final_kernel(const uint32_t* __restrict__ in,
                                                              const uint32_t* __restrict__ gather,
                                                              size_t n,
                                                              const uint32_t* __restrict__ parts,
                                                              uint32_t* __restrict__ out) {
  scan_final_body<GATHER, INCLUSIVE>(in, gather, n, parts, out, blockIdx.x);
}

// Lanes of this wave whose digit equals mine (among lanes with valid == true).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid, int bits) {
  uint64_t m = __ballot(valid);
  for (int b = 0; b < bits; b++) {
    const bool set = (d >> b) & 1u;
    const uint64_t bal = __ballot(set);
    m &= set ? bal : ~bal;
  }
  return valid ? m : 0ull;
}

// ---- one-sweep LSD radix sort ---------------------------------------------------------------------
// Per sort: one memset (digit totals, partition tickets, look-back status), one launch computing
// the digit totals of EVERY pass from the unsorted keys (a permutation does not change them), and
// one launch per 8-bit pass that ranks, scans and scatters in a single sweep:
//   * a workgroup takes a ticket (atomic counter) = its partition of kSortTile keys, so every
//     partition it may wait for belongs to a workgroup that is already running;
//   * it ranks its keys stably (wave64 ballot "match" of the digit, per-wave running counts in
//     LDS), publishes its per-digit counts as AGGREGATE, then each thread (= one digit) walks back
//     over the predecessors' status words until an INCLUSIVE prefix, and publishes its own
//     INCLUSIVE prefix (decoupled look-back);
//   * the keys are re-ordered in LDS by digit and written out in runs, so that consecutive lanes
//     store consecutive addresses of one digit bucket.
// Status word (u64): bits 32-33 flag (0 = not yet published, 1 = aggregate, 2 = inclusive),
// bits 0-31 count.  Polling is bounded: after kSpinLimit empty polls a thread gives up, raises
// the error word (checked by the host at its next synchronisation) and proceeds, so no wave can
// hang the device.
constexpr uint64_t kStAgg = 1ull << 32, kStIncl = 2ull << 32, kStFlags = 3ull << 32;
constexpr uint64_t kStOne = 1ull << 32;  // one contributor in a super-partition word
}  // namespace
// count of timed-out look-backs since the last check (sort_timeouts_word)
__device__ uint32_t g_lookback_timeouts;
// test hook (gsr_test_force_sort_timeout): every look-back behaves as if its spin bound ran out
__device__ uint32_t g_force_lookback_timeout;
// Sticky per-device fault word (kStatus* bits of every failed forward since the last
// gsr_reset_forward_faults): set by the tile-ranges kernel and the forward blend; the fused Adam
// step reads it and leaves the parameters and moments untouched while it is non-zero, so NaN
// gradients of a failed call never reach them (the reference __trap()s, auxiliary.h:156-160).
__device__ uint32_t g_forward_faults;
namespace {
constexpr int kSpinLimit = 1 << 18;
// One-sweep workgroup size: NT lanes share a partition of kSortTile keys.  More lanes keep the
// ranking chain short (kSortTile / NT keys per lane) and hide its LDS latency with other waves
// (256 lanes = one wave per SIMD, every latency exposed: 7.5 us of ranking per pass); but 1024-lane
// workgroups (48 KB LDS, 16 waves) fit only 2 per CU, so with more than 2 x 256 partitions the
// late ones wait for a slot.  1024 lanes when every partition is resident at once, else 512.
constexpr uint32_t kResident1024 = 2 * 256;  // 1024-lane partitions resident at once (256 CUs)

// Digit totals of every pass from the unsorted keys.  Its own tile (kTotKPT keys per thread) and a
// bounded grid striding over tiles: short per-workgroup chains for latency, and at most
// kTotGroups global atomics per counter at the end.
constexpr int kTotKPT = 8;
constexpr size_t kTotGroups = 1024;
constexpr int kTotTile = kThreads * kTotKPT;

__host__ __device__ __forceinline__ int sort_digit_width(int bits) { return sort_digit_bits(bits); }

// (body shared by the one-sort kernel and the several-sorts kernel: blk / nblk = this
// workgroup's index and the workgroup count of its sort)
__device__ __forceinline__ void radix_totals_body(const uint32_t* __restrict__ keys, size_t n,
                                                  int bits, uint32_t* __restrict__ totals,
                                                  uint32_t* __restrict__ nsent_out,
                                                  int skip_sentinel, uint32_t blk, uint32_t nblk,
                                                  int lo = 0) {
  __shared__ uint32_t cnt[kSortMaxPasses][256];
  __shared__ uint32_t nsent;  // sentinel keys of this workgroup (all digits 0xff)
#pragma unroll
  for (int p = 0; p < kSortMaxPasses; p++) cnt[p][threadIdx.x] = 0;
  if (threadIdx.x == 0) nsent = 0;
  __syncthreads();
  const int passes = (bits + 7) / 8;
  const int dw = sort_digit_width(bits);
  const uint32_t dmask = (1u << dw) - 1u;
  for (size_t base = (size_t)blk * kTotTile; base < n; base += (size_t)nblk * kTotTile) {
    // all loads of the tile in flight before any is consumed
    uint32_t key[kTotKPT];
#pragma unroll
    for (int r = 0; r < kTotKPT; r++) {
      const size_t i = base + (size_t)r * kThreads + threadIdx.x;
      key[r] = i < n ? keys[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < kTotKPT; r++) {
      const bool valid = base + (size_t)r * kThreads + threadIdx.x < n;
      const uint64_t vmask = __ballot(valid);
      if (vmask == 0ull) continue;
      if (skip_sentinel) {
        const uint64_t sm = __ballot(valid && key[r] == kSortSentinel);
        if (sm && (threadIdx.x & 63) == 0) atomicAdd(&nsent, (uint32_t)__popcll(sm));
      }
      for (int p = 0; p < passes; p++) {
        const uint32_t d = (key[r] >> (lo + dw * p)) & dmask;
        // typical depth keys share their top byte across a wave: one LDS add instead of 64
        // serialised same-address atomics
        const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
        if (__ballot(valid && d != d0) == 0ull) {
          if ((threadIdx.x & 63) == 0) atomicAdd(&cnt[p][d0], (uint32_t)__popcll(vmask));
        } else if (valid) {
          atomicAdd(&cnt[p][d], 1u);
        }
      }
    }
  }
  __syncthreads();
  // this workgroup's partial copy of the totals (see kSortTotShards)
  const uint32_t shard = blk % (uint32_t)kSortTotShards;
  uint32_t* tot = totals + (size_t)shard * kSortMaxPasses * 256;
  for (int p = 0; p < passes; p++) {
    const uint32_t c = cnt[p][threadIdx.x];
    if (c) atomicAdd(&tot[p * 256 + threadIdx.x], c);
  }
  if (threadIdx.x == 0 && nsent) atomicAdd(&nsent_out[shard], nsent);
}

// Planned sort (radix_sort_pairs kc): one workgroup per sort, after the totals launch, writes the
// plan -- bit p set for each pass whose digit is not the same for every non-sentinel key (the
// passes that run); none: the last pass runs (a copy that places the result and gathers the
// payload).  (A separate launch: a last-workgroup plan inside the totals launch needs an
// agent-scope release fence per workgroup, an L2 write-back each.)
__device__ __forceinline__ void sort_plan_body(const uint32_t* __restrict__ aux, int bits,
                                               int skip_sentinel, uint32_t* __restrict__ plan_out) {
  __shared__ uint32_t s_n[kSortMaxPasses][kThreads / 64];
  const int passes = (bits + 7) / 8;
  const int dw = sort_digit_width(bits);
  uint32_t sent = 0;
  if (skip_sentinel) {
#pragma unroll
    for (int sh = 0; sh < kSortTotShards; sh++) sent += aux[kSortAuxSent + sh];
  }
  for (int p = 0; p < passes; p++) {
    const int dbits = (bits - dw * p) < dw ? (bits - dw * p) : dw;
    const uint32_t dig = threadIdx.x;  // kThreads = 256 digits
    uint32_t c = 0;
    if (dig < (1u << dbits)) {
#pragma unroll
      for (int sh = 0; sh < kSortTotShards; sh++)
        c += aux[kSortAuxTotals + (size_t)sh * kSortMaxPasses * 256 + p * 256 + dig];
      // sentinel keys (every digit at its maximum) do not count
      if (dig == (1u << dbits) - 1u) c -= sent;
    }
    const uint64_t b = __ballot(c != 0u);
    if ((threadIdx.x & 63) == 0) s_n[p][threadIdx.x >> 6] = (uint32_t)__popcll(b);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t plan = 0;
    for (int p = 0; p < passes; p++)
      if (s_n[p][0] + s_n[p][1] + s_n[p][2] + s_n[p][3] > 1u) plan |= 1u << p;
    if (plan == 0) plan = 1u << (passes - 1);
    plan_out[0] = plan;
  }
}

__global__ __launch_bounds__(kThreads) void sort_plan_kernel(uint32_t* __restrict__ aux, int bits,
                                                             int skip_sentinel) {
  sort_plan_body(aux, bits, skip_sentinel, aux + kSortAuxPlan);
}

__global__ __launch_bounds__(kThreads) void radix_totals_kernel(const uint32_t* __restrict__ keys,
                                                                size_t n, int bits,
                                                                uint32_t* __restrict__ totals,
                                                                uint32_t* __restrict__ nsent_out,
                                                                int skip_sentinel) {
  radix_totals_body(keys, n, bits, totals, nsent_out, skip_sentinel, blockIdx.x, gridDim.x);
}

// The buffers of pass `pass` of a planned sort (radix_sort_pairs kc): the passes that run (plan
// bits) read (ka, va) first and alternate so that the last one writes (kb, vb).  False: this pass
// does not run.
struct PassBufs {
  const uint32_t *kin, *vin;
  uint32_t *kout, *vout;
  bool last;
};
__device__ __forceinline__ bool planned_pass(uint32_t plan, int pass, const uint32_t* ka,
                                             const uint32_t* va, uint32_t* kb, uint32_t* vb,
                                             uint32_t* kc, uint32_t* vc, PassBufs& o) {
  if (!((plan >> pass) & 1u)) return false;
  const int k = __popc(plan), j = __popc(plan & ((1u << pass) - 1u));
  // run j writes B when (k - 1 - j) is even, else C; it reads what run j - 1 wrote (A for j = 0)
  const bool out_b = ((k - 1 - j) & 1) == 0;
  o.kout = out_b ? kb : kc;
  o.vout = out_b ? vb : vc;
  o.kin = j == 0 ? ka : (out_b ? kc : kb);
  o.vin = j == 0 ? va : (out_b ? vc : vb);
  o.last = j == k - 1;
  return true;
}

__device__ __forceinline__ uint64_t status_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void status_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NT>
__device__ __forceinline__ void onesweep_body(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, size_t n, int shift,
    int bits, const uint32_t* __restrict__ totals, const uint32_t* __restrict__ nsent_sh,
    uint32_t* __restrict__ ticket, uint64_t* __restrict__ status, uint32_t* __restrict__ err,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, const uint32_t* __restrict__ kpay,
    uint32_t blk, uint32_t nblk, uint32_t ulo = 0, uint32_t vsplit = 0) {
  constexpr int kSortWaves = NT / 64, kSortThreads = NT;
  // Keys-only sort (vin null, grid-uniform): packed keys whose low bits carry the value; the
  // last pass (ulo > 0) writes them out as the pair (key >> ulo, key & (2^ulo - 1)), earlier
  // passes the packed key alone (vout null).
  // One sorted element out at position o: its value, and its key -- or (last pass) the payload
  // gathered by its value, kpay[v]
  // (vsplit: the values carry the payload in their high bits -- the last pass splits them)
  auto emit = [&](uint32_t o, uint32_t v, uint32_t k) {
    if (vsplit) {
      kout[o] = v >> vsplit;
      vout[o] = v & ((1u << vsplit) - 1u);
      return;
    }
    if (ulo) {
      kout[o] = k >> ulo;
      vout[o] = k & ((1u << ulo) - 1u);
      return;
    }
    kout[o] = kpay ? kpay[min(v, (uint32_t)n - 1u)] : k;
    if (vout) vout[o] = v;
  };
  constexpr int kKeysPerThread = kSortTile / NT, kKeysPerWave = kKeysPerThread * 64;
  static_assert(NT >= 256 && kSortTile % NT == 0, "one-sweep tile shape");
  __shared__ uint32_t s_k[kSortTile];
  __shared__ uint32_t s_v[kSortTile];
  __shared__ uint32_t s_cnt[kSortWaves][256];
  __shared__ uint32_t s_gofs[256];
  __shared__ uint32_t s_scan[kSortWaves];
  __shared__ uint32_t s_part;
  const int t = (int)threadIdx.x, lane = t & 63, wid = t >> 6;
  const uint32_t mask = (1u << bits) - 1u;
  // thread t < 2^bits <-> digit t: this pass's digit total, summed over the partial copies (a
  // narrower last digit -- 4 bits for 3024 tiles -- publishes and looks back 16 words per
  // partition instead of 256)
  const bool dig = t < (1 << bits);
  const int dt = dig ? t : 0;
  uint32_t dtotal = 0;
  if (dig) {
#pragma unroll
    for (int sh = 0; sh < kSortTotShards; sh++) dtotal += totals[(size_t)sh * kSortMaxPasses * 256 + t];
  }
  {
    // Every non-sentinel key has the same digit in this pass: the stable sort by it is the
    // identity on those keys, and sentinel keys may land anywhere -- the pass is a copy (no
    // ranking, no look-back).  Workgroup-uniform (the totals are final before the launch).
    uint32_t real = dtotal;
    if (t == 255 && nsent_sh) {
#pragma unroll
      for (int sh = 0; sh < kSortTotShards; sh++) real -= nsent_sh[sh];
    }
    const uint64_t b = __ballot(dig && real != 0u);
    if (lane == 0 && wid < 4) s_scan[wid] = (uint32_t)__popcll(b);
    __syncthreads();
    const uint32_t ndig = s_scan[0] + s_scan[1] + s_scan[2] + s_scan[3];
    if (ndig <= 1u) {
      const size_t b0 = (size_t)blk * kSortTile;
      const size_t e0 = min(n, b0 + (size_t)kSortTile);
      for (size_t i = b0 + (size_t)t; i < e0; i += NT) emit((uint32_t)i, vin ? vin[i] : 0u, kin[i]);
      return;
    }
  }
  // ticket, not blockIdx: a partition can only wait on partitions whose workgroups already run
  // (a per-XCD ticket variant timed out its look-back on gfx950 -- dispatch order across XCDs
  // gives no such guarantee)
#if GSR_SORT_TICKET
  if (t == 0) s_part = atomicAdd(ticket, 1u);
#else
  // blockIdx order: every XCD dispatches its workgroups in index order, so the lowest unfinished
  // partition is always resident and the look-back always progresses (bounded spin as backstop)
  if (t == 0) s_part = blk;
#endif
  for (int e = t; e < kSortWaves * 256; e += kSortThreads) (&s_cnt[0][0])[e] = 0;
  __syncthreads();
  const uint32_t part = s_part;
  const size_t base = (size_t)part * kSortTile;
  const size_t wbase = base + (size_t)wid * kKeysPerWave;

  uint32_t key[kKeysPerThread], val[kKeysPerThread];
#pragma unroll
  for (int r = 0; r < kKeysPerThread; r++) {
    const size_t i = wbase + (size_t)r * 64 + lane;
    key[r] = i < n ? kin[i] : 0u;
    val[r] = (vin && i < n) ? vin[i] : 0u;
  }
  // stable rank inside the wave's 1024 consecutive keys
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint32_t rk[kKeysPerThread];
#pragma unroll
  for (int r = 0; r < kKeysPerThread; r++) {
    const bool valid = wbase + (size_t)r * 64 + lane < n;
    const uint32_t d = (key[r] >> shift) & mask;
    const uint64_t peers = match_digit(d, valid, bits);
    const uint32_t before = s_cnt[wid][d];
    rk[r] = before + (uint32_t)__popcll(peers & lt);
    if (valid && (__ffsll((long long)peers) - 1) == lane) s_cnt[wid][d] = before + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  // (the lanes t >= 256 join the workgroup scans with zeros)
  uint32_t h = 0;
  if (dig)
#pragma unroll
    for (int w = 0; w < kSortWaves; w++) h += s_cnt[w][t];
  uint64_t* my = status + (size_t)part * 256 + dt;
  // super-partition words follow the partition words of this pass (sort_pass_words)
  uint64_t* super = status + (size_t)nblk * 256;
  if (dig) {
    status_store(my, (part == 0 ? kStIncl : kStAgg) | (uint64_t)h);
    // one contributor and its count into the super-partition's word: self-describing (complete
    // when the contributor count reaches kSortSuper), so no fence orders it against other words
    __hip_atomic_fetch_add(super + (size_t)(part / kSortSuper) * 256 + dt, kStOne | (uint64_t)h,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  uint32_t total_n;
  const uint32_t lstart = block_excl_scan<kSortWaves>(dig ? h : 0u, s_scan, total_n);
  const uint32_t dbase = block_excl_scan<kSortWaves>(dig ? dtotal : 0u, s_scan, total_n);
  if (dig) {
    uint32_t run = lstart;
#pragma unroll
    for (int w = 0; w < kSortWaves; w++) {
      const uint32_t c = s_cnt[w][t];
      s_cnt[w][t] = run;
      run += c;
    }
  }
  __syncthreads();
  // keys to their digit-ordered slots in LDS now, before the look-back: the local order does not
  // depend on the global offsets, and the look-back then runs with the keys out of registers
  // (75 VGPRs at 512 lanes: 3 workgroups per CU, so 768 partitions are resident at once)
#pragma unroll
  for (int r = 0; r < kKeysPerThread; r++) {
    if (wbase + (size_t)r * 64 + lane < n) {
      const uint32_t d = (key[r] >> shift) & mask;
      const uint32_t pos = s_cnt[wid][d] + rk[r];
      s_k[pos] = key[r];
      if (vin) s_v[pos] = val[r];
    }
  }
  uint32_t excl = 0;
  if (dig && part > 0) {
    // Two-level windowed look-back.  (A) the predecessors inside this partition's own
    // super-partition (at most kSortSuper - 1 words, 8 per round), consumed in order up to the
    // first INCLUSIVE word or the first word not yet published (re-polled from there).  (B) then
    // whole super-partitions, newest first, 4 at a time: the inclusive word of a
    // super-partition's last partition ends the walk, else its super word once complete (all
    // kSortSuper contributors) adds its 16 partitions at once.  Partition 0 is always INCLUSIVE,
    // so the walk ends at super-partition 0 at the latest.  A look-back crosses 16x fewer
    // unpublished-prefix words than a partition-by-partition walk (the frontier of inclusive
    // prefixes advances 256 partitions per round instead of 16).
    int spins = 0;
    bool done = false;
    auto spin = [&]() {
      if (++spins > kSpinLimit) {
        atomicOr(err, 1u);
        atomicAdd(&g_lookback_timeouts, 1u);  // sticky, read back by every forward
        done = true;
        return;
      }
      // fail fast: once any partition of this sort gave up, the others stop waiting too (a
      // predecessor that never publishes would otherwise cost every later partition its own
      // full spin bound in turn -- minutes of apparent hang instead of one bound)
      if ((spins & 63) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        done = true;
        return;
      }
      __builtin_amdgcn_s_sleep(1);
    };
    if (g_force_lookback_timeout) {  // test hook only: the bounded spin's give-up path
      atomicOr(err, 1u);
      atomicAdd(&g_lookback_timeouts, 1u);
      done = true;
    }
    const int64_t qlo = (int64_t)(part / kSortSuper) * kSortSuper;
    int64_t q = (int64_t)part - 1;
    constexpr int kAW = 8;  // partition words per round inside the super-partition (no spill)
    while (!done && q >= qlo) {
      uint64_t w[kAW];
#pragma unroll
      for (int j = 0; j < kAW; j++)
        w[j] = (q - j >= qlo) ? status_load(status + (size_t)(q - j) * 256 + dt) : 0ull;
      int used = 0;
      bool stop = false;
#pragma unroll
      for (int j = 0; j < kAW; j++) {  // branch-free so that w[] stays in registers
        const uint64_t f = w[j] & kStFlags;
        const bool take = !stop && q - j >= qlo && f != 0;
        excl += take ? (uint32_t)w[j] : 0u;
        used = take ? j + 1 : used;
        done = done || (take && f == kStIncl);
        stop = stop || !take || f == kStIncl;
      }
      q -= used;
      if (!done && q >= qlo && used < kAW) spin();  // stopped at a word not yet published
    }
    int64_t S = (int64_t)(part / kSortSuper) - 1;
    constexpr int kSW = 4;  // super-partitions per round (8 loads in flight per digit: no spill)
    while (!done && S >= 0) {
      uint64_t lw[kSW], sw[kSW];
#pragma unroll
      for (int j = 0; j < kSW; j++) {
        const bool in = S - j >= 0;
        lw[j] = in ? status_load(status + (size_t)((S - j) * kSortSuper + kSortSuper - 1) * 256 + dt)
                   : 0ull;
        sw[j] = in ? status_load(super + (size_t)(S - j) * 256 + dt) : 0ull;
      }
      int used = 0;
      bool stop = false;
#pragma unroll
      for (int j = 0; j < kSW; j++) {
        const bool in = S - j >= 0;
        const bool incl = in && (lw[j] & kStFlags) == kStIncl;
        const bool full = in && (uint32_t)(sw[j] >> 32) == (uint32_t)kSortSuper;
        const bool take = !stop && (incl || full);
        excl += take ? (uint32_t)(incl ? lw[j] : sw[j]) : 0u;
        used = take ? j + 1 : used;
        done = done || (take && incl);
        stop = stop || !take || incl;
      }
      S -= used;
      if (!done && S >= 0 && used < kSW) spin();  // stopped at an incomplete super-partition
    }
    status_store(my, kStIncl | (uint64_t)(excl + h));
  }
  if (dig) s_gofs[t] = dbase + excl - lstart;
  __syncthreads();
  const uint32_t nvalid = (uint32_t)min((size_t)kSortTile, n - base);
  for (uint32_t i = (uint32_t)t; i < nvalid; i += kSortThreads) {
    const uint32_t k = s_k[i];
    const uint32_t o = s_gofs[(k >> shift) & mask] + i;
    if (o < n) emit(o, vin ? s_v[i] : 0u, k);  // only a timed-out look-back (error word raised) can produce o >= n
  }
}

template <int NT>
__global__ __launch_bounds__(NT, NT == 1024 ? 8 : (NT == 512 ? 6 : 1)) void radix_onesweep_kernel(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, size_t n, int shift,
    int bits, const uint32_t* __restrict__ totals, const uint32_t* __restrict__ nsent_sh,
    uint32_t* __restrict__ ticket, uint64_t* __restrict__ status, uint32_t* __restrict__ err,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, const uint32_t* __restrict__ kpay) {
  onesweep_body<NT>(kin, vin, n, shift, bits, totals, nsent_sh, ticket, status, err, kout, vout,
                    kpay, blockIdx.x, gridDim.x);
}

// a pass of a planned sort: (kin, vin) = A, (kout, vout) = B, (kc, vc) = C; plan = kSortAuxPlan
template <int NT>
__global__ __launch_bounds__(NT, NT == 1024 ? 8 : (NT == 512 ? 6 : 1)) void radix_planned_kernel(
    const uint32_t* __restrict__ ka, const uint32_t* __restrict__ va, size_t n, int pass,
    int shift, int bits, const uint32_t* __restrict__ totals, const uint32_t* __restrict__ nsent_sh,
    uint32_t* __restrict__ ticket, uint64_t* __restrict__ status, uint32_t* __restrict__ err,
    uint32_t* __restrict__ kb, uint32_t* __restrict__ vb, uint32_t* __restrict__ kc,
    uint32_t* __restrict__ vc, const uint32_t* __restrict__ kpay, const uint32_t* plan) {
  PassBufs o;
  if (!planned_pass(*plan, pass, ka, va, kb, vb, kc, vc, o)) return;  // grid-uniform
  onesweep_body<NT>(o.kin, o.vin, n, shift, bits, totals, nsent_sh, ticket, status, err, o.kout,
                    o.vout, o.last ? kpay : nullptr, blockIdx.x, gridDim.x);
}

// ---- several independent sorts / scans / sums per launch (the multi-view forward's batched
// binning).  Workgroup b belongs to view k with first[k] <= b < first[k + 1] (workgroup-uniform);
// inside a view everything is exactly the one-view kernel: its own digit totals, tickets and
// look-back words, so the views never wait on each other and each result is bit-identical to its
// own one-view sort.
struct SortPassJob {
  const uint32_t* kin;
  const uint32_t* vin;
  uint32_t* kout;
  uint32_t* vout;
  uint32_t *kc, *vc;     // planned sort: (kin, vin) = A, (kout, vout) = B, this = C (else null)
  const uint32_t* kpay;  // last pass: payload gathered in place of the key
  uint32_t* aux;         // totals, sentinel counts, tickets, error word (kSortAux*)
  const uint32_t* tot;   // the digit totals the passes read (aux's, or SortSpec::totals)
  uint64_t* status;      // this pass's look-back words
  uint32_t n;
  uint32_t ulo;          // keys-only sort, last pass: the value bits to unpack (else 0)
  uint32_t vsplit;       // last pass: split the values at this bit (else 0; SortSpec::vsplit)
};
struct SortPassViews {
  SortPassJob j[kMaxBatchViews];
  uint32_t first[kMaxBatchViews + 1];
  int V;
};

__device__ __forceinline__ int batch_view(const uint32_t* first, int V, uint32_t b) {
  int k = 0;
  while (k + 1 < V && b >= first[k + 1]) k++;
  return k;
}

struct SumJob {
  const uint32_t* parts;
  const uint32_t* parts2;
  uint32_t* out;
  uint32_t* host;
  const uint32_t* flag0;
  int n;
};
struct SumViews {
  SumJob j[kMaxBatchViews];
  int V;
};
// one view's read-back sums (exact and full-rectangle instance counts, sticky flag) by one
// workgroup of NT lanes
template <int NT>
__device__ __forceinline__ void sum_job_body(const SumJob& j) {
  __shared__ uint32_t lds[NT / 64], lds2[NT / 64];
  uint32_t s = 0, s2 = 0;
  for (int i = (int)threadIdx.x; i < j.n; i += NT) {
    s += j.parts[i];
    s2 += j.parts2[i];
  }
  uint32_t total, total2;
  block_excl_scan<NT / 64>(s, lds, total);
  block_excl_scan<NT / 64>(s2, lds2, total2);
  if (threadIdx.x == 0) {
    j.out[0] = total;
    j.out[1] = total2;
    if (j.host) {
      j.host[0] = j.flag0 ? *j.flag0 : 0u;
      j.host[1] = total;
      j.host[2] = total2;
    }
  }
}

// sm.V > 0: each view's first workgroup also forms that view's read-back sums (the launch that
// would otherwise do it alone, one workgroup per view, is folded in here)
__global__ __launch_bounds__(kThreads) void radix_totals_views_kernel(SortPassViews m, int bits,
                                                                      int skip_sentinel, int lo,
                                                                      SumViews sm) {
  const int k = batch_view(m.first, m.V, blockIdx.x);
  const SortPassJob& j = m.j[k];
  if (sm.V && blockIdx.x == m.first[k]) sum_job_body<kThreads>(sm.j[k]);
  radix_totals_body(j.kin, j.n, bits, j.aux + kSortAuxTotals, j.aux + kSortAuxSent, skip_sentinel,
                    blockIdx.x - m.first[k], m.first[k + 1] - m.first[k], lo);
}

// one workgroup per view (planned sorts)
__global__ __launch_bounds__(kThreads) void sort_plan_views_kernel(SortPassViews m, int bits,
                                                                   int skip_sentinel) {
  const SortPassJob& j = m.j[blockIdx.x];
  if (j.n == 0) return;
  sort_plan_body(j.aux, bits, skip_sentinel, j.aux + kSortAuxPlan);
}

template <int NT>
__global__ __launch_bounds__(NT, NT == 1024 ? 8 : (NT == 512 ? 6 : 1)) void radix_onesweep_views_kernel(
    SortPassViews m, int pass, int shift, int bits, int sentinel) {
  const int k = batch_view(m.first, m.V, blockIdx.x);
  const SortPassJob& j = m.j[k];
  PassBufs o{j.kin, j.vin, j.kout, j.vout, true};
  if (j.kc) {  // planned (workgroup-uniform per view: the view's own plan)
    if (!planned_pass(j.aux[kSortAuxPlan], pass, j.kin, j.vin, j.kout, j.vout, j.kc, j.vc, o)) return;
  }
  onesweep_body<NT>(o.kin, o.vin, j.n, shift, bits, j.tot + 256 * pass,
                    sentinel ? j.aux + kSortAuxSent : nullptr, j.aux + kSortAuxTickets + 8 * pass,
                    j.status, j.aux + kSortAuxErr, o.kout, o.vout, o.last ? j.kpay : nullptr,
                    blockIdx.x - m.first[k], m.first[k + 1] - m.first[k], j.ulo,
                    o.last ? j.vsplit : 0u);
}

struct ScanJob {
  const uint32_t* in;
  uint32_t* out;
  uint32_t* parts;
  uint32_t n;
};
struct ScanViews {
  ScanJob j[kMaxBatchViews];
  uint32_t first[kMaxBatchViews + 1];
  int V;
};

__global__ __launch_bounds__(kThreads) void scan_reduce_views_kernel(ScanViews m) {
  const int k = batch_view(m.first, m.V, blockIdx.x);
  const ScanJob& j = m.j[k];
  scan_reduce_body<false>(j.in, nullptr, j.n, j.parts, blockIdx.x - m.first[k]);
}

// RAW (each workgroup sums its predecessors' plain partials itself) reads O(parts^2) words in
// total, so it is taken only up to kScanRawMaxParts partitions per view; above, one workgroup per
// view scans the partials first (scan_parts_views_kernel) and the final pass reads its prefix.
constexpr uint32_t kScanRawMaxParts = 1024;

__global__ __launch_bounds__(1024) void scan_parts_views_kernel(ScanViews m) {
  const int k = (int)blockIdx.x;
  scan_parts_body(m.j[k].parts, (int)(m.first[k + 1] - m.first[k]));
}

template <bool INCLUSIVE, bool RAW>
__global__ __launch_bounds__(kThreads) void scan_final_views_kernel(ScanViews m) {
  const int k = batch_view(m.first, m.V, blockIdx.x);
  const ScanJob& j = m.j[k];
  scan_final_body<false, INCLUSIVE, RAW>(j.in, nullptr, j.n, j.parts, j.out,
                                         blockIdx.x - m.first[k]);
}

// One workgroup: *out = sum of the n partials (n <= kScanMaxParts).
// out[0] = sum of parts[0..n); with parts2: out[1] = sum of parts2[0..n) (the forward's exact
// instance count and the reference's full-rectangle count, gsr_api.cpp, one read-back for both).
__global__ __launch_bounds__(1024) void sum_parts_kernel(const uint32_t* __restrict__ parts, int n,
                                                         uint32_t* __restrict__ out,
                                                         const uint32_t* __restrict__ parts2) {
  __shared__ uint32_t lds[16], lds2[16];
  uint32_t s = 0, s2 = 0;
  for (int i = (int)threadIdx.x; i < n; i += 1024) {
    s += parts[i];
    if (parts2) s2 += parts2[i];
  }
  uint32_t total, total2 = 0;
  block_excl_scan<16>(s, lds, total);
  if (parts2) block_excl_scan<16>(s2, lds2, total2);  // kernel-argument (uniform) branch
  if (threadIdx.x == 0) {
    out[0] = total;
    if (parts2) out[1] = total2;
  }
}

// ---- single-pass inclusive scan with decoupled look-back, several views per launch -------------
// One launch instead of scan_u32's three (reduce, one-workgroup partials scan, final): a
// workgroup takes a ticket (its partition of kScanTile elements), scans it, publishes the
// aggregate, and wave 0 walks back over the predecessors' status words 64 at a time until an
// inclusive prefix (u64 words as the sort's: bits 32-33 flag, 0-31 count).  Bounded polling: a
// timed-out look-back raises `err` (the depth sort's error word: the forward's status check
// reports it) and the partition proceeds.  In the batched forward the one-workgroup middle pass
// of scan_u32 waited ~80 us for a dispatch slot behind the other group's duplication.
struct ScanLbJob {
  const uint32_t* in;
  uint32_t* out;
  uint64_t* st;  // [0]: ticket counter; [1 + p]: partition p's status (zeroed before the launch)
  uint32_t* err;
  uint32_t n;
};
struct ScanLbViews {
  ScanLbJob j[kMaxBatchViews];
  uint32_t first[kMaxBatchViews + 1];
  int V;
};

__global__ __launch_bounds__(kThreads) void scan_lookback_views_kernel(ScanLbViews m) {
  __shared__ uint32_t lds[kThreads / 64];
  __shared__ uint32_t s_part, s_prefix;
  int k = 0;
  while (k + 1 < m.V && blockIdx.x >= m.first[k + 1]) k++;  // workgroup-uniform
  const ScanLbJob& job = m.j[k];
  const int t = (int)threadIdx.x, lane = t & 63;
  if (t == 0) s_part = atomicAdd(reinterpret_cast<uint32_t*>(job.st), 1u);
  __syncthreads();
  const uint32_t p = s_part;
  const size_t base = (size_t)p * kScanTile + (size_t)t * kScanItems;
  uint32_t v[kScanItems];
  uint32_t sum = 0;
#pragma unroll
  for (int q = 0; q < kScanItems; q++) {
    const size_t i = base + q;
    v[q] = i < job.n ? job.in[i] : 0u;
    sum += v[q];
  }
  uint32_t total;
  const uint32_t excl = block_excl_scan<kThreads / 64>(sum, lds, total);
  uint64_t* st = job.st + 1;
  if (t == 0) status_store(st + p, (p == 0 ? kStIncl : kStAgg) | (uint64_t)total);
  if (p > 0 && t < 64) {
    uint32_t prefix = 0;
    int64_t q = (int64_t)p - 1;
    int spins = 0;
    while (q >= 0) {
      const int64_t src = q - lane;
      const uint64_t w = src >= 0 ? status_load(st + src) : kStIncl;  // before partition 0: done
      const uint64_t f = w & kStFlags;
      const uint64_t incl = __ballot(f == kStIncl);
      const uint64_t ready = __ballot(f != 0);
      // lanes up to and including the first inclusive word (all of them if none is inclusive)
      const int upto = incl ? __ffsll((long long)incl) - 1 : 63;
      const uint64_t need = upto >= 63 ? ~0ull : ((2ull << upto) - 1ull);
      if ((ready & need) == need) {
        uint32_t x = (lane <= upto && src >= 0) ? (uint32_t)w : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x += (uint32_t)__shfl_xor((int)x, d, 64);
        prefix += x;
        if (incl) break;
        q -= 64;
        continue;
      }
      if (++spins > kSpinLimit || g_force_lookback_timeout) {  // bounded: report and proceed
        if (lane == 0) {
          atomicOr(job.err, 1u);
          atomicAdd(&g_lookback_timeouts, 1u);
        }
        break;
      }
      // fail fast once another partition gave up (see the sort's spin)
      if ((spins & 63) == 0 && __hip_atomic_load(job.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) {
      status_store(st + p, kStIncl | (uint64_t)(prefix + total));
      s_prefix = prefix;
    }
  }
  __syncthreads();
  uint32_t run = (p == 0 ? 0u : s_prefix) + excl;
#pragma unroll
  for (int q = 0; q < kScanItems; q++) {
    const size_t i = base + q;
    run += v[q];
    if (i < job.n) job.out[i] = run;
  }
}

// One workgroup per view: out = {sum parts, sum parts2}; host (device-mapped pinned words, may be
// null) = {*flag0, the two sums}: the views' read-back is these stores plus one event, no copy.
__global__ __launch_bounds__(1024) void sum_parts_views_kernel(SumViews m) {
  sum_job_body<1024>(m.j[blockIdx.x]);
}
}  // namespace

hipError_t sum_u32_parts_views(const SumSpec* v, int V, hipStream_t s) {
  if (V <= 0) return hipSuccess;
  if (V > kMaxBatchViews) return hipErrorInvalidValue;
  SumViews m{};
  m.V = V;
  for (int k = 0; k < V; k++) {
    if (v[k].n > 0x7fffffffull || !v[k].parts2) return hipErrorInvalidValue;
    m.j[k] = SumJob{v[k].parts, v[k].parts2, v[k].out, v[k].host, v[k].flag0, (int)v[k].n};
  }
  hipLaunchKernelGGL(sum_parts_views_kernel, dim3((unsigned)V), dim3(1024), 0, s, m);
  return hipGetLastError();
}

hipError_t scan_u32_lookback_views(const ScanLbSpec* v, int V, hipStream_t s) {
  if (V <= 0) return hipSuccess;
  if (V > kMaxBatchViews) return hipErrorInvalidValue;
  ScanLbViews m{};
  m.V = V;
  m.first[0] = 0;
  for (int k = 0; k < V; k++) {
    if (v[k].n > 0xffffffffull) return hipErrorInvalidValue;
    m.j[k] = ScanLbJob{v[k].in, v[k].out, v[k].status, v[k].err, (uint32_t)v[k].n};
    m.first[k + 1] = m.first[k] + (uint32_t)scan_parts(v[k].n);
  }
  if (m.first[V] == 0) return hipSuccess;
  hipLaunchKernelGGL(scan_lookback_views_kernel, dim3(m.first[V]), dim3(kThreads), 0, s, m);
  return hipGetLastError();
}

hipError_t scan_u32_views(const ScanSpec* v, int V, bool inclusive, hipStream_t s) {
  if (V <= 0) return hipSuccess;
  if (V > kMaxBatchViews) return hipErrorInvalidValue;
  ScanViews m{};
  m.V = V;
  m.first[0] = 0;
  size_t np_max = 0;
  for (int k = 0; k < V; k++) {
    const size_t np = scan_parts(v[k].n);
    if (np > (size_t)kScanMaxParts || v[k].n > 0xffffffffull) return hipErrorInvalidValue;
    m.j[k] = ScanJob{v[k].in, v[k].out, v[k].parts, (uint32_t)v[k].n};
    m.first[k + 1] = m.first[k] + (uint32_t)np;
    np_max = np > np_max ? np : np_max;
  }
  if (m.first[V] == 0) return hipSuccess;
  const dim3 grid(m.first[V]);
  const bool raw = np_max <= kScanRawMaxParts;
  hipLaunchKernelGGL(scan_reduce_views_kernel, grid, dim3(kThreads), 0, s, m);
  if (!raw) hipLaunchKernelGGL(scan_parts_views_kernel, dim3(V), dim3(1024), 0, s, m);
  if (raw) {
    if (inclusive) hipLaunchKernelGGL((scan_final_views_kernel<true, true>), grid, dim3(kThreads), 0, s, m);
    else hipLaunchKernelGGL((scan_final_views_kernel<false, true>), grid, dim3(kThreads), 0, s, m);
  } else {
    if (inclusive) hipLaunchKernelGGL((scan_final_views_kernel<true, false>), grid, dim3(kThreads), 0, s, m);
    else hipLaunchKernelGGL((scan_final_views_kernel<false, false>), grid, dim3(kThreads), 0, s, m);
  }
  return hipGetLastError();
}

hipError_t sum_u32_parts(const uint32_t* parts, size_t n, uint32_t* out, hipStream_t s,
                         const uint32_t* parts2) {
  if (n > 0x7fffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(1024), 0, s, parts, (int)n, out, parts2);
  return hipGetLastError();
}

hipError_t reduce_u32(const uint32_t* in, size_t n, uint32_t* parts, uint32_t* out,
                      hipStream_t s) {
  if (n == 0) return hipMemsetAsync(out, 0, sizeof(uint32_t), s);
  const size_t np = scan_parts(n);
  if (np > (size_t)kScanMaxParts) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scan_reduce_kernel<false>, dim3((unsigned)np), dim3(kThreads), 0, s, in,
                     (const uint32_t*)nullptr, n, parts);
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(1024), 0, s, parts, (int)np, out,
                     (const uint32_t*)nullptr);
  return hipGetLastError();
}

hipError_t scan_u32(const uint32_t* in, const uint32_t* gather, uint32_t* out, size_t n,
                    bool inclusive, uint32_t* parts, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const size_t np = scan_parts(n);
  if (np > (size_t)kScanMaxParts) return hipErrorInvalidValue;
  const dim3 grid((unsigned)np);
  if (gather) hipLaunchKernelGGL(scan_reduce_kernel<true>, grid, dim3(kThreads), 0, s, in, gather, n, parts);
  else hipLaunchKernelGGL(scan_reduce_kernel<false>, grid, dim3(kThreads), 0, s, in, gather, n, parts);
  hipLaunchKernelGGL(scan_parts_kernel, dim3(1), dim3(1024), 0, s, parts, (int)np);
  if (gather) {
    if (inclusive) hipLaunchKernelGGL((scan_final_kernel<true, true>), grid, dim3(kThreads), 0, s, in, gather, n, parts, out);
    else hipLaunchKernelGGL((scan_final_kernel<true, false>), grid, dim3(kThreads), 0, s, in, gather, n, parts, out);
  } else {
    if (inclusive) hipLaunchKernelGGL((scan_final_kernel<false, true>), grid, dim3(kThreads), 0, s, in, gather, n, parts, out);
    else hipLaunchKernelGGL((scan_final_kernel<false, false>), grid, dim3(kThreads), 0, s, in, gather, n, parts, out);
  }
  return hipGetLastError();
}


extern "C" int gsr_test_force_sort_timeout(int on) {
  const uint32_t v = on ? 1u : 0u;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_force_lookback_timeout), &v, sizeof(v)) == hipSuccess ? 0 : 2;
}

uint32_t* forward_faults_word() {
  // the symbol's address on the current device, looked up once per device
  constexpr int kMaxDev = 64;
  static std::atomic<uint32_t*> cache[kMaxDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  uint32_t* w = cache[dev].load(std::memory_order_relaxed);
  if (w) return w;
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_forward_faults)) != hipSuccess) return nullptr;
  cache[dev].store((uint32_t*)p, std::memory_order_relaxed);
  return (uint32_t*)p;
}

extern "C" int gsr_forward_faults(void) {
  uint32_t v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_forward_faults), sizeof(v)) != hipSuccess) return -1;
  return (int)v;
}

extern "C" int gsr_reset_forward_faults(void) {
  const uint32_t v = 0;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_forward_faults), &v, sizeof(v)) == hipSuccess ? 0 : 2;
}

uint32_t* sort_timeouts_word() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_lookback_timeouts)) != hipSuccess) return nullptr;
  return (uint32_t*)p;
}

hipError_t radix_sort_pairs(uint32_t* ka, uint32_t* va, uint32_t* kb, uint32_t* vb, size_t n,
                            int bits, SortScratch scratch, bool* result_in_b, hipStream_t s,
                            bool sentinel_anywhere, bool precleared,
                            const uint32_t* key_payload, uint32_t* kc, uint32_t* vc) {
  *result_in_b = false;
  if (kc && !vc) return hipErrorInvalidValue;
  if (n == 0 || bits <= 0) return hipSuccess;
  if (bits > 32 || n > 0xffffffffull) return hipErrorInvalidValue;
  const int passes = sort_passes(bits);
  const uint32_t nb = (uint32_t)sort_blocks(n);
  // aux (totals, tickets, error word) and the status words of the passes used: one memset
  if (!precleared) {
    hipError_t e = hipMemsetAsync(scratch.aux, 0, sort_clear_bytes(scratch, n, bits), s);
    if (e != hipSuccess) return e;
  }
  const size_t tot_tiles = (n + kTotTile - 1) / kTotTile;
  hipLaunchKernelGGL(radix_totals_kernel,
                     dim3((unsigned)(tot_tiles < kTotGroups ? tot_tiles : kTotGroups)),
                     dim3(kThreads), 0, s, ka, n, bits, scratch.aux + kSortAuxTotals,
                     scratch.aux + kSortAuxSent, sentinel_anywhere ? 1 : 0);
  if (kc)
    hipLaunchKernelGGL(sort_plan_kernel, dim3(1), dim3(kThreads), 0, s, scratch.aux, bits,
                       sentinel_anywhere ? 1 : 0);
  uint32_t *kin = ka, *vin = va, *kout = kb, *vout = vb;
  bool in_b = false;
  for (int p = 0; p < passes; p++) {
    const int dw = sort_digit_width(bits);
    const int shift = dw * p;
    const int dbits = (bits - shift) < dw ? (bits - shift) : dw;
    const int nt = nb <= kResident1024 ? 1024 : 512;
    if (kc) {  // planned: the pass itself reads the plan and picks its buffers
#define GSR_PLANNED(NT)                                                                           \
  hipLaunchKernelGGL(radix_planned_kernel<NT>, dim3(nb), dim3(NT), 0, s, ka, va, n, p, shift,    \
                     dbits, scratch.aux + kSortAuxTotals + 256 * p,                              \
                     sentinel_anywhere ? scratch.aux + kSortAuxSent : nullptr,                   \
                     scratch.aux + kSortAuxTickets + 8 * p,                                      \
                     scratch.status + (size_t)p * sort_pass_words(n), scratch.aux + kSortAuxErr, \
                     kb, vb, kc, vc, key_payload, scratch.aux + kSortAuxPlan)
      if (nt == 1024) GSR_PLANNED(1024);
      else GSR_PLANNED(512);
#undef GSR_PLANNED
      continue;
    }
#define GSR_ONESWEEP(NT)                                                                          \
  hipLaunchKernelGGL(radix_onesweep_kernel<NT>, dim3(nb), dim3(NT), 0, s, kin, vin, n, shift,    \
                     dbits, scratch.aux + kSortAuxTotals + 256 * p,                              \
                     sentinel_anywhere ? scratch.aux + kSortAuxSent : nullptr,                   \
                     scratch.aux + kSortAuxTickets + 8 * p,                                      \
                     scratch.status + (size_t)p * sort_pass_words(n), \
                     scratch.aux + kSortAuxErr, kout, vout,                                      \
                     p == passes - 1 ? key_payload : nullptr)
    if (nt == 1024) GSR_ONESWEEP(1024);
    else GSR_ONESWEEP(512);
#undef GSR_ONESWEEP
    uint32_t* t;
    t = kin; kin = kout; kout = t;
    t = vin; vin = vout; vout = t;
    in_b = !in_b;
  }
  *result_in_b = kc ? true : in_b;
  return hipGetLastError();
}

}  // namespace gsr

namespace gsr {

hipError_t radix_sort_pairs_views(const SortSpec* v, int V, int bits, bool* result_in_b,
                                  hipStream_t s, bool sentinel_anywhere, bool precleared,
                                  const SumSpec* sums, hipEvent_t after_totals) {
  *result_in_b = false;
  if (V <= 0 || bits <= 0) return hipSuccess;
  if (V > kMaxBatchViews || bits > 32) return hipErrorInvalidValue;
  const int passes = sort_passes(bits);
  SortPassViews m{};
  m.V = V;
  const bool planned = v[0].kc != nullptr;
  // keys-only packed sort (SortSpec::lo): every view or none, not planned, no payload gather
  const int lo = v[0].lo;
  if (lo < 0 || lo + bits > 32 || (lo && planned)) return hipErrorInvalidValue;
  for (int k = 0; k < V; k++)
    if (v[k].lo != lo || (lo && v[k].key_payload) || v[k].vsplit < 0 || v[k].vsplit >= 32 ||
        (v[k].vsplit && (v[k].key_payload || lo)))
      return hipErrorInvalidValue;
  // totals formed upstream (the multi-view duplication): no totals launch
  const bool given = v[0].totals != nullptr;
  if (given && (planned || sums || after_totals || sentinel_anywhere)) return hipErrorInvalidValue;
  uint32_t tfirst[kMaxBatchViews + 1] = {0}, ofirst[kMaxBatchViews + 1] = {0};
  for (int k = 0; k < V; k++) {
    const size_t n = v[k].n;
    if ((v[k].totals != nullptr) != given) return hipErrorInvalidValue;
    if (n > 0xffffffffull) return hipErrorInvalidValue;
    if ((v[k].kc != nullptr) != planned || (v[k].kc && !v[k].vc)) return hipErrorInvalidValue;
    if (!precleared && n) {
      hipError_t e = hipMemsetAsync(v[k].scratch.aux, 0, sort_clear_bytes(v[k].scratch, n, bits), s);
      if (e != hipSuccess) return e;
    }
    const size_t tt = (n + kTotTile - 1) / kTotTile;
    tfirst[k + 1] = tfirst[k] + (uint32_t)(tt < kTotGroups ? tt : kTotGroups);
    ofirst[k + 1] = ofirst[k] + (uint32_t)sort_blocks(n);
  }
  if (ofirst[V] == 0) return hipSuccess;
  auto fill = [&](int p, const uint32_t* first) {
    for (int k = 0; k <= V; k++) m.first[k] = first[k];
    // pass p reads the pair written by pass p - 1; planned: (A, B, C), each pass picks its own
    const bool b_in = !planned && (p & 1) != 0;
    for (int k = 0; k < V; k++) {
      const SortSpec& w = v[k];
      SortPassJob& j = m.j[k];
      const bool last = p == passes - 1;
      j.kin = b_in ? w.kb : w.ka;
      j.vin = lo ? nullptr : (b_in ? w.vb : w.va);
      j.kout = (b_in && !planned) ? w.ka : w.kb;
      j.vout = (lo && !last) ? nullptr : ((b_in && !planned) ? w.va : w.vb);
      j.ulo = (lo && last) ? (uint32_t)lo : 0u;
      j.kc = w.kc;
      j.vc = w.vc;
      j.kpay = (planned || p == passes - 1) ? w.key_payload : nullptr;
      j.vsplit = (planned || p == passes - 1) ? (uint32_t)w.vsplit : 0u;
      j.aux = w.scratch.aux;
      j.tot = w.totals ? w.totals : w.scratch.aux + kSortAuxTotals;
      j.status = w.scratch.status + (size_t)p * sort_pass_words(w.n);
      j.n = (uint32_t)w.n;
    }
  };
  fill(0, tfirst);
  SumViews sm{};
  if (sums) {  // one per view, in the views' order
    sm.V = V;
    for (int k = 0; k < V; k++) {
      if (sums[k].n > 0x7fffffffull || !sums[k].parts2) return hipErrorInvalidValue;
      sm.j[k] = SumJob{sums[k].parts, sums[k].parts2, sums[k].out, sums[k].host, sums[k].flag0,
                       (int)sums[k].n};
    }
  }
  if (!given)
    hipLaunchKernelGGL(radix_totals_views_kernel, dim3(tfirst[V]), dim3(kThreads), 0, s, m, bits,
                       sentinel_anywhere ? 1 : 0, lo, sm);
  if (after_totals) {
    const hipError_t e = hipEventRecord(after_totals, s);
    if (e != hipSuccess) return e;
  }
  if (planned)
    hipLaunchKernelGGL(sort_plan_views_kernel, dim3(V), dim3(kThreads), 0, s, m, bits,
                       sentinel_anywhere ? 1 : 0);
  const uint32_t nb = ofirst[V];
  const int nt = nb <= kResident1024 ? 1024 : 512;
  for (int p = 0; p < passes; p++) {
    fill(p, ofirst);
    const int dw = sort_digit_width(bits);
    const int shift = dw * p;
    const int dbits = (bits - shift) < dw ? (bits - shift) : dw;
    if (nt == 1024)
      hipLaunchKernelGGL(radix_onesweep_views_kernel<1024>, dim3(nb), dim3(1024), 0, s, m, p,
                         lo + shift, dbits, sentinel_anywhere ? 1 : 0);
    else
      hipLaunchKernelGGL(radix_onesweep_views_kernel<512>, dim3(nb), dim3(512), 0, s, m, p,
                         lo + shift, dbits, sentinel_anywhere ? 1 : 0);
  }
  *result_in_b = planned || (passes & 1) != 0;
  return hipGetLastError();
}

}  // namespace gsr
