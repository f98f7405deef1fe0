// RetinaNet inference (retinanet.py:285-387) in four launches on gfx950:
// per level the exact top_k(sigmoid(logits), topk_candidates, sorted=True)
// (TF TopKV2: value desc, ties lowest index first), the score threshold, the
// box decode, then per image the class-offset NMS (NonMaxSuppressionV3) over
// the concatenated levels and the zero padding.
//
//   floor    one workgroup per (image, level) segment: samples one 1,024-key
//            run out of every 128 K keys, takes the sampled key that about
//            4 k keys of the segment reach (bitonic sort of the threads'
//            sample maxima) and lowers it to the lowest raw key with the same
//            sigmoid.  Segments of <= 8,192 keys take every key.
//   collect  one pass over every score (the only full read: 4 B per score),
//            a persistent grid with the next chunk's loads in flight while
//            the current one is tested.  No atomics: each wave of each chunk
//            owns 8 candidate slots and a count it always writes; only the
//            hits past a wave's 8 slots take an atomic on the segment's
//            overflow buffer (device-scope atomics on one address serialize
//            across the 8 XCDs: one per hitting wave cost 350 us here).
//   finish   one workgroup per segment: gathers the slots; they are exact
//            when at least k of them lie at or above the floor's sigmoid edge
//            (every key below the floor then has a smaller sigmoid) and
//            nothing overflowed; otherwise the workgroup selects exactly
//            (radix passes over the segment, then the sigmoid tie group in
//            index order).  Sort keys (sigmoid desc, index asc); the k-th
//            smallest by a radix select in registers, the <= 1,024 keys at or
//            below it bitonic-sorted with in-wave exchanges; threshold,
//            decode of the kept top-k, the per-image max coordinate.
//   nms      one workgroup per image: merge rank of the per-level sorted
//            lists (binary searches in lockstep; the concat position breaks
//            ties), then greedy NMS of the class-offset boxes in 64-candidate
//            tiles against the kept list, stopping at max_detections -- the
//            full candidate x candidate mask of nms.hip is never built.
//
// Exact in every case (the floor only decides how often the in-workgroup
// select runs); the tie rules, sigmoid, IoU and decode expressions are those
// of the unfused pipeline (topk.hip, nms.hip, proposals.hip), which stays
// selectable with the tuning key "retina_fused" = 0.
#include "detect.h"

namespace d2mi {
namespace {

constexpr int kWG = 1024;                 // per-segment / per-image workgroups
constexpr int kCap = kLdsSortCap;         // candidates per segment
constexpr int kRun = 1024;                // sampled run (keys)
constexpr int kRunStride = 131072;        // one run per 128 K keys
constexpr int kCT = 256;                  // collect threads
constexpr int kCW = kCT / 64;             // collect waves
constexpr int kCV = 4;                    // float4 per collect thread per chunk
constexpr int kChunk4 = kCT * kCV;        // float4 per chunk (16 KB)
constexpr int kWaveSlots = 8;             // candidate slots per (chunk, wave)
constexpr int kTile = 64;                 // NMS tile
constexpr int kRankWin = 128;             // NMS window ranked in the NMS workgroup (retina_var 4096)
constexpr int kPT = 1024;                 // compact: wave slots per part (one per thread)
constexpr int kPartCap = kPT * kWaveSlots;  // compact: entries a part can hold

struct SegInfo {
  uint32_t floor;     // collect keys >= floor
  uint32_t exact_lo;  // keys >= exact_lo have a larger sigmoid than any key < floor
  int32_t k;          // effective k: min(topk_candidates, anchors, keys)
  int32_t exact;      // 1: skip the floor, select in the workgroup (tests)
  int32_t novf;       // collect's overflow appends (counted past kCap)
  int32_t pad;
  uint64_t ts[10];    // wall-clock stamps of the phases (tools/retina_post_ab.py --debug)
  uint64_t cyc[10];   // shader-clock stamps at the same points (the clock the phases ran at)
  uint64_t sub[8];    // stamps inside the sort (4) and the NMS (4) phases (tools/retina_post_ab.py)
};

struct RetinaGeo {
  int32_t len[D2MI_MAX_LEVELS];         // keys per image and level (H W A K)
  int32_t anchors[D2MI_MAX_LEVELS];     // H W A
  int32_t chunk0[D2MI_MAX_LEVELS + 1];  // per-image prefix of collect chunks
  int32_t L, N, K;
  int32_t part0[D2MI_MAX_LEVELS + 1];   // per-image prefix of compact parts (kPT wave slots each)
};

__device__ __forceinline__ const float* seg_ptr(const float* base, const Levels& lv, int n, int l,
                                                int K) {
  return base + lv.off_a[l] + (int64_t)n * lv.img_a[l] * K;
}

__device__ __forceinline__ uint64_t stamp() { return (uint64_t)wall_clock64(); }
__device__ __forceinline__ uint64_t cycles() { return (uint64_t)clock64(); }

// Wave-aggregated append: one atomic per wave with hits.  Returns the slot
// of this lane's hit (or -1).  Lanes outside the branch do not take part.
__device__ __forceinline__ int wave_append(bool hit, int* counter) {
  const uint64_t b = __ballot(hit);
  if (!b) return -1;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)b) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(b));
  base = __shfl(base, leader);
  return hit ? base + __popcll(b & ((1ull << lane) - 1ull)) : -1;
}

// Inclusive scan of one value across the wave in DPP row shifts and row
// broadcasts (no LDS crossbar round trips): within rows of 16, then row 15
// into rows 1 and 3, then lane 31 into rows 2 and 3.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

// Inclusive scan of one value per thread over the workgroup (part: 16 words).
__device__ __forceinline__ uint32_t wg_inclusive_scan(uint32_t v, uint32_t* part, bool dpp = false) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = v;
  if (dpp) {
    incl = wave_incl_scan_dpp(v);
  } else {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
  }
  if (lane == 63) part[w] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (int j = 0; j < w; ++j) before += part[j];
  __syncthreads();
  return before + incl;
}

// Bitonic sort of 1,024 keys, one per thread; returns the key at the thread's
// position in ascending order.  Exchanges at strides < 64 stay in the wave
// (cross-lane), the 10 larger ones go through lds (2 x 1,024 words, used in
// turn: one barrier per exchange).
__device__ uint64_t bitonic1024(uint64_t v, uint64_t* lds) {
  const int t = threadIdx.x;
  int buf = 0;
  auto step = [&](int size, int stride) {
    uint64_t o;
    if (stride < 64) {
      o = (uint64_t)__shfl_xor((unsigned long long)v, stride);
    } else {
      uint64_t* b = lds + buf * kWG;
      b[t] = v;
      __syncthreads();
      o = b[t ^ stride];
      buf ^= 1;
    }
    const bool up = (t & size) == 0, low = (t & stride) == 0;
    const uint64_t mn = v < o ? v : o, mx = v < o ? o : v;
    v = (low == up) ? mn : mx;
  };
  for (int size = 2; size <= kWG; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) step(size, stride);
  return v;
}

// The same sort with the exchanges at strides < 64 done in VALU lane
// permutations (tuning retina_var 128): DPP quad / row / half-row mirrors for
// strides 1 - 8, v_permlane16_swap / v_permlane32_swap (gfx950) for 16 and
// 32 -- no LDS crossbar round trip and no address arithmetic -- and the
// compare-exchange as one 64-bit compare and a select; fully unrolled.  The
// shuffle form runs ~25 VALU per stage per wave, which at 16 waves per CU is
// what bound it (11.5 us for 55 stages, profiles/r6s_retina_post_ab.log).
template <int S>
__device__ __forceinline__ uint32_t lane_xor32(uint32_t v) {
  if constexpr (S == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  } else if constexpr (S == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
  } else if constexpr (S == 4) {  // half-row mirror (p ^ 7), then quad reverse (p ^ 3)
    const int h = __builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_mov_dpp(h, 0x1B, 0xF, 0xF, false);
  } else if constexpr (S == 8) {  // row mirror (p ^ 15), then half-row mirror (p ^ 7)
    const int m = __builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_mov_dpp(m, 0x141, 0xF, 0xF, false);
  } else if constexpr (S == 16) {  // odd rows of the first operand <-> even rows of the second
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return ((threadIdx.x >> 4) & 1) ? r[0] : r[1];
  } else {  // S == 32: upper half of the first operand <-> lower half of the second
    static_assert(S == 32, "lane_xor32: strides 1 - 32");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return ((threadIdx.x >> 5) & 1) ? r[0] : r[1];
  }
}

template <int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic_strides(uint64_t& v, uint64_t* lds, int& buf) {
  const int t = threadIdx.x;
  uint64_t o;
  if constexpr (STRIDE >= 64) {
    uint64_t* b = lds + buf * kWG;
    b[t] = v;
    __syncthreads();
    o = b[t ^ STRIDE];
    buf ^= 1;
  } else {
    o = ((uint64_t)lane_xor32<STRIDE>((uint32_t)(v >> 32)) << 32) | lane_xor32<STRIDE>((uint32_t)v);
  }
  const bool want_min = ((t & SIZE) == 0) == ((t & STRIDE) == 0);
  // (branch-free: take the partner's key when it is on the wanted side; on
  // equal keys either choice is the same key)
  v = ((o < v) == want_min) ? o : v;
  if constexpr (STRIDE > 1) bitonic_strides<SIZE, STRIDE / 2>(v, lds, buf);
}
template <int SIZE>
__device__ __forceinline__ void bitonic_sizes(uint64_t& v, uint64_t* lds, int& buf) {
  bitonic_strides<SIZE, SIZE / 2>(v, lds, buf);
  if constexpr (SIZE < kWG) bitonic_sizes<SIZE * 2>(v, lds, buf);
}
__device__ __forceinline__ uint64_t bitonic1024_lanes(uint64_t v, uint64_t* lds) {
  int buf = 0;
  bitonic_sizes<2>(v, lds, buf);
  return v;
}

// ------------------------------------------------------------------ floor
__global__ __launch_bounds__(kWG) void retina_floor_kernel(const float* __restrict__ base,
                                                           Levels lv, RetinaGeo g, int topk,
                                                           int force_exact, int radix,
                                                           int spread,
                                                           SegInfo* __restrict__ info,
                                                           uint32_t* __restrict__ maxc) {
  const uint64_t t_start = stamp(), c_start = cycles();
  const int s = blockIdx.x, n = s / g.L, l = s - n * g.L;
  const int len = g.len[l];
  const int kk = max(0, min(min(topk, g.anchors[l]), len));
  const int t = threadIdx.x;
  __shared__ uint64_t xch[kWG];
  __shared__ uint32_t s_floor;
  if (l == 0 && t == 0) maxc[n] = kKeyNegInf;
  if (kk == 0 || len <= kCap || force_exact) {
    if (t == 0) {
      info[s].floor = kk == 0 ? 0xffffffffu : 0u;
      info[s].exact_lo = 0u;
      info[s].k = kk;
      info[s].exact = (kk > 0 && len > kCap && force_exact) ? 1 : 0;
      info[s].novf = 0;
      info[s].ts[0] = t_start;
      info[s].ts[1] = stamp();
      info[s].cyc[0] = c_start;
      info[s].cyc[1] = cycles();
    }
    return;
  }
  const float* p = seg_ptr(base, lv, n, l, g.K);
  const int nruns = (len + kRunStride - 1) / kRunStride;
  uint32_t best = 0;
  if ((((uintptr_t)p) & 15) == 0 && nruns >= 8) {
    // every run but the last is whole: thread t takes float4 (t & 255) of runs
    // (t >> 8) + 4 u, 24 loads in flight (one round for up to 96 runs)
    constexpr int U = 24;
    const int q = t & 255, full = nruns - 1;
    for (int r0 = t >> 8; r0 < full; r0 += 4 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + 4 * u;
        v[u] = r < full ? *reinterpret_cast<const float4*>(p + (int64_t)r * kRunStride + 4 * q)
                        : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        best = max(best, max(max(orderable(v[u].x), orderable(v[u].y)),
                             max(orderable(v[u].z), orderable(v[u].w))));
    }
    const int64_t e = (int64_t)full * kRunStride + t;  // the last run, one key per thread
    if (e < len) best = max(best, orderable(p[e]));
  } else if (spread) {
    // (few runs, retina_var 2) the same number of samples,
    // spread evenly over the whole segment: on a model's outputs the first
    // 1,024 keys of a small level are one or two anchor positions, and P7's
    // floor from them left 9,969 keys above it -- past the candidate buffer,
    // so the exact select ran (44 us on the critical path)
    int64_t ns = 0;
    for (int r = 0; r < nruns; ++r) ns += min<int64_t>(kRun, len - (int64_t)r * kRunStride);
    const int64_t stride = max<int64_t>(1, len / ns);
    for (int r = 0; r < nruns; ++r) {
      const int64_t i = (int64_t)r * kRun + t;
      if (i < ns) best = max(best, orderable(p[i * stride]));
    }
  } else {  // (few runs: one sample per thread and run, so the maxima are the samples)
    for (int r = 0; r < nruns; ++r) {
      const int64_t e = (int64_t)r * kRunStride + t;
      if (e < len) best = max(best, orderable(p[e]));
    }
  }
  int64_t nsamp = 0;
  for (int r = 0; r < nruns; ++r) nsamp += min<int64_t>(kRun, len - (int64_t)r * kRunStride);
  // keys of the whole segment at the floor: about 4 k (never past the
  // candidate buffer's middle ground), as a count of sampled keys
  const int target = min(4 * kk, (kk + kCap) / 2);
  const int ts = (int)max<int64_t>(1, min<int64_t>(kWG, (int64_t)target * nsamp / len));
  // the ts-th largest thread maximum, bit by bit from the top (the largest
  // value that at least ts maxima reach), by wave 0 alone: ballot counts, no
  // further barriers
  __shared__ uint32_t mx[kWG];
  uint32_t f0 = 0;
  if (radix) {
    // (retina_var 8192) the same value -- the ts-th largest maximum with its
    // low 8 bits cleared -- by a radix select over the whole workgroup: three
    // 8-bit passes of LDS histogram atomics, each bin searched from the top by
    // wave 0 (4 bins per lane, one DPP scan), instead of wave 0's 24 rounds
    // of 16 compare-ballots
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_pref, s_krem;
    if (t == 0) {
      s_pref = 0;
      s_krem = (uint32_t)ts;
    }
    for (int pass = 0; pass < 3; ++pass) {
      const int sh = 24 - 8 * pass;
      if (t < 256) hist[t] = 0;
      __syncthreads();
      const uint32_t pref = s_pref;
      if (pass == 0 || (best >> (sh + 8)) == pref) atomicAdd(&hist[(best >> sh) & 255u], 1u);
      __syncthreads();
      if (t < 64) {
        const uint32_t krem = s_krem;
        uint32_t c4[4], loc = 0;  // lane t: bins 255 - 4t .. 252 - 4t
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          c4[j] = hist[255 - (4 * t + j)];
          loc += c4[j];
        }
        const uint32_t incl = wave_incl_scan_dpp(loc);
        const uint64_t hitm = __ballot(incl >= krem);
        const int first = hitm ? __ffsll((unsigned long long)hitm) - 1 : 63;
        if (t == first) {
          uint32_t acc = incl - loc;
          int bin = 252 - 4 * t;
          for (int j = 0; j < 4; ++j) {
            if (acc + c4[j] >= krem) {
              bin = 255 - (4 * t + j);
              break;
            }
            acc += c4[j];
          }
          s_pref = (pref << 8) | (uint32_t)bin;
          s_krem = krem - acc;
        }
      }
      __syncthreads();
    }
    f0 = s_pref << 8;
    if (t >= 64) return;
  } else {
  mx[t] = best;
  __syncthreads();
  if (t >= 64) return;
  // (the top 24 bits only: the floor is a heuristic, a key at most 255
  // steps lower collects a few more candidates and changes no result)
  {
    uint32_t vals[kWG / 64];
#pragma unroll
    for (int j = 0; j < kWG / 64; ++j) vals[j] = mx[j * 64 + t];
    for (int b = 31; b >= 8; --b) {
      const uint32_t cand = f0 | (1u << b);
      int c = 0;
#pragma unroll
      for (int j = 0; j < kWG / 64; ++j) c += __popcll(__ballot(vals[j] >= cand));
      if (c >= ts) f0 = cand;
    }
  }
  }
  uint32_t floor = f0, exact_lo = f0;
  if (f0 > kKeyNegInf && f0 <= kKeyPosInf) {  // no sigmoid tie across exact_lo
    const uint32_t lb = wave_lower_bound_sig(kKeyNegInf, f0, sigmoidf_tf(from_orderable(f0)));
    exact_lo = lb;
    floor = lb > kKeyNegInf + kWindowMargin ? lb - kWindowMargin : kKeyNegInf;
  }
  if (t == 0) {
    info[s].floor = floor;
    info[s].exact_lo = exact_lo;
    info[s].k = kk;
    info[s].exact = 0;
    info[s].novf = 0;
    info[s].ts[0] = t_start;
    info[s].ts[1] = stamp();
    info[s].cyc[0] = c_start;
    info[s].cyc[1] = cycles();
  }
}

// ---------------------------------------------------------------- collect
struct ChunkAt {
  const float4* p4;
  int s, h, len, q0, n4;
  uint32_t floor;
  bool on;
};

__device__ __forceinline__ ChunkAt locate_chunk(int c, const float* base, const Levels& lv,
                                                const RetinaGeo& g, const SegInfo* info) {
  const int cpi = g.chunk0[g.L];
  const int n = c / cpi, r = c - n * cpi;
  int l = 0;
  while (l + 1 < g.L && g.chunk0[l + 1] <= r) ++l;
  ChunkAt a;
  a.s = n * g.L + l;
  const float* p = seg_ptr(base, lv, n, l, g.K);
  a.h = (int)(((uintptr_t)p >> 2) & 3);
  a.p4 = reinterpret_cast<const float4*>(p - a.h);
  a.len = g.len[l];
  a.n4 = (a.h + a.len + 3) >> 2;
  a.q0 = (r - g.chunk0[l]) * kChunk4;
  a.floor = info[a.s].floor;
  a.on = info[a.s].k > 0 && !info[a.s].exact && a.q0 < a.n4;
  return a;
}

typedef float nv4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void load_chunk(const ChunkAt& a, float4 (&v)[kCV]) {
  const nv4* p = reinterpret_cast<const nv4*>(a.p4);
#pragma unroll
  for (int u = 0; u < kCV; ++u) {
    const int q = a.q0 + u * kCT + threadIdx.x;
    nv4 x = {0.f, 0.f, 0.f, 0.f};
    if (a.on && q < a.n4) x = __builtin_nontemporal_load(&p[q]);  // read once: no reuse
    v[u] = make_float4(x.x, x.y, x.z, x.w);
  }
}

__global__ __launch_bounds__(kCT) void retina_collect_kernel(
    const float* __restrict__ base, Levels lv, RetinaGeo g, SegInfo* __restrict__ info,
    int32_t* __restrict__ wcount, uint64_t* __restrict__ wslot, uint64_t* __restrict__ ovf) {
  const int total = g.N * g.chunk0[g.L];
  int c = blockIdx.x;
  if (c >= total) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  ChunkAt cur = locate_chunk(c, base, lv, g, info);
  float4 v[kCV];
  load_chunk(cur, v);
  for (; c < total; c += gridDim.x) {
    const int cn = c + gridDim.x;
    ChunkAt nxt = cur;
    float4 w[kCV];
    if (cn < total) {
      nxt = locate_chunk(cn, base, lv, g, info);
      load_chunk(nxt, w);
    }
    auto hit = [&](int q, int i, float e) {
      return cur.on && q < cur.n4 && i >= 0 && i < cur.len && orderable(e) >= cur.floor;
    };
    int cnt = 0;
#pragma unroll
    for (int u = 0; u < kCV; ++u) {
      const int q = cur.q0 + u * kCT + threadIdx.x;
      const int i0 = 4 * q - cur.h;
      cnt += (hit(q, i0, v[u].x) ? 1 : 0) + (hit(q, i0 + 1, v[u].y) ? 1 : 0) +
             (hit(q, i0 + 2, v[u].z) ? 1 : 0) + (hit(q, i0 + 3, v[u].w) ? 1 : 0);
    }
    const size_t slot = (size_t)c * kCW + wv;
    if (__ballot(cnt > 0)) {
      int incl = cnt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      const int wtot = __shfl(incl, 63);
      int ob = 0;  // this wave's first overflow position (hits past its 8 slots)
      if (wtot > kWaveSlots) {
        if (lane == 0) ob = atomicAdd(&info[cur.s].novf, wtot - kWaveSlots);
        ob = __shfl(ob, 0);
      }
      if (lane == 0) wcount[slot] = wtot;
      int pos = incl - cnt;
      // entry-major: entry j of every slot in one row (the gather reads first
      // entries contiguously)
      const size_t nslots = (size_t)total * kCW;
      uint64_t* dst = wslot + slot;
      uint64_t* odst = ovf + (size_t)cur.s * kCap;
#pragma unroll
      for (int u = 0; u < kCV; ++u) {
        const int q = cur.q0 + u * kCT + threadIdx.x;
        const int i0 = 4 * q - cur.h;
        const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (hit(q, i0 + j, e[j])) {
            const uint64_t ent = ((uint64_t)__float_as_uint(e[j]) << 32) | (uint32_t)(i0 + j);
            if (pos < kWaveSlots) dst[(size_t)pos * nslots] = ent;
            else if (ob + pos - kWaveSlots < kCap) odst[ob + pos - kWaveSlots] = ent;
            ++pos;
          }
        }
      }
    } else if (lane == 0) {
      wcount[slot] = 0;
    }
    cur = nxt;
#pragma unroll
    for (int u = 0; u < kCV; ++u) v[u] = w[u];
  }
}

// ---------------------------------------------------------------- compact
// (tuning retina_var 16) Many workgroups per segment: part p of segment s
// compacts the slot entries of kPT wave slots into its own region (no
// atomics, so nothing to zero first) and writes its count; the finish then
// gathers ~k x 4 contiguous entries instead of every wave slot's count.
__global__ __launch_bounds__(kPT) void retina_compact_kernel(RetinaGeo g,
                                                             const int32_t* __restrict__ wcount,
                                                             const uint64_t* __restrict__ wslot,
                                                             uint64_t* __restrict__ cand,
                                                             int32_t* __restrict__ pcnt) {
  const int s = blockIdx.y, n = s / g.L, l = s - n * g.L;
  const int part = blockIdx.x;
  if (part >= g.part0[l + 1] - g.part0[l]) return;
  __shared__ uint32_t sp[kPT / 64];
  const int t = threadIdx.x;
  const int cpi = g.chunk0[g.L];
  const int w0 = (n * cpi + g.chunk0[l]) * kCW;
  const int nw = (g.chunk0[l + 1] - g.chunk0[l]) * kCW;
  const size_t nslots = (size_t)g.N * cpi * kCW;
  const int e = part * kPT + t;
  const int slot = w0 + min(e, nw - 1);
  const int c = e < nw ? min(wcount[slot], kWaveSlots) : 0;
  const uint64_t e1 = wslot[slot];  // (loaded with the count: a slot's rows always exist)
  const uint32_t incl = wg_inclusive_scan((uint32_t)c, sp);
  const int pos = (int)incl - c;
  const int gp = n * g.part0[g.L] + g.part0[l] + part;
  uint64_t* dst = cand + (size_t)gp * kPartCap;
  if (c > 0) dst[pos] = e1;
  for (int j = 1; j < c; ++j) dst[pos + j] = wslot[(size_t)j * nslots + slot];
  if (t == kPT - 1) pcnt[gp] = (int)incl;
}

// ----------------------------------------------------------------- finish
// f(index, value) over a segment by the whole workgroup: aligned float4 body
// (8 loads in flight per thread), scalar head and tail.
template <typename F>
__device__ __forceinline__ void wg_visit(const float* __restrict__ p, int len, F f) {
  const int h = min(len, (int)((4 - (((uintptr_t)p >> 2) & 3)) & 3));
  if ((int)threadIdx.x < h) f((int)threadIdx.x, p[threadIdx.x]);
  const float4* p4 = reinterpret_cast<const float4*>(p + h);
  const int n4 = (len - h) >> 2;
  constexpr int U = 8;
  for (int q0 = 0; q0 < n4; q0 += U * kWG) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u * kWG + threadIdx.x;
      v[u] = q < n4 ? p4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u * kWG + threadIdx.x;
      if (q < n4) {
        const int i = h + 4 * q;
        f(i, v[u].x);
        f(i + 1, v[u].y);
        f(i + 2, v[u].z);
        f(i + 3, v[u].w);
      }
    }
  }
  const int t0 = h + 4 * n4;
  if (t0 + (int)threadIdx.x < len) f(t0 + (int)threadIdx.x, p[t0 + threadIdx.x]);
}

// The exact top-k set of p[0, len) by (sigmoid desc, index asc) into sk as
// raw entries (value bits << 32 | index); returns their count (k, or more
// when the tie group fits: the sort orders ties by index).  Radix select of
// the k-th largest raw key u (12 + 12 + 8 bits), then keys above u's sigmoid
// tie group and the group itself (keys of equal sigmoid, tested exactly in a
// window below it), the group in index order when it does not fit.
__device__ int exact_select(const float* __restrict__ p, int len, int k, uint64_t* sk,
                            uint32_t* hist, uint32_t* part, int32_t* err) {
  __shared__ int s_bin;
  __shared__ uint32_t s_gt;
  __shared__ int s_above, s_tie;
  __shared__ uint32_t s_tie_hi, s_win_lo;
  __shared__ float s_sig;
  __shared__ int s_sigmode;
  const int t = threadIdx.x;
  uint32_t prefix = 0;
  int krem = k;
  for (int pass = 0; pass < 3; ++pass) {
    const int nbits = pass < 2 ? 12 : 8;
    const int shift = pass == 0 ? 20 : (pass == 1 ? 8 : 0);
    const int hs = shift + nbits;
    const uint32_t mask = (1u << nbits) - 1u;
    for (int i = t; i < 4096; i += kWG) hist[i] = 0;
    if (t == 0) s_bin = -1;
    __syncthreads();
    wg_visit(p, len, [&](int, float v) {
      const uint32_t key = orderable(v);
      if (hs == 32 || (key >> hs) == prefix) atomicAdd(&hist[(key >> shift) & mask], 1u);
    });
    __syncthreads();
    // thread t owns 4 bins from the top: 4095 - 4t .. 4092 - 4t
    uint32_t c4[4], loc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c4[j] = hist[4095 - (4 * t + j)];
      loc += c4[j];
    }
    const uint32_t incl = wg_inclusive_scan(loc, part);
    const uint32_t before = incl - loc;
    if ((uint32_t)krem > before && (uint32_t)krem <= incl) {
      uint32_t acc = before;
      for (int j = 0; j < 4; ++j) {
        if ((uint32_t)krem <= acc + c4[j]) {
          s_bin = 4095 - (4 * t + j);
          s_gt = acc;
          break;
        }
        acc += c4[j];
      }
    }
    __syncthreads();
    if (s_bin < 0) {  // counts inconsistent (cannot happen)
      if (t == 0) atomicOr(err, kErrTopkCapacity);
      return 0;
    }
    prefix = (prefix << nbits) | (uint32_t)s_bin;
    krem -= (int)s_gt;
    __syncthreads();
  }
  const uint32_t u = prefix;
  if (t < 64) {  // (wave 0: the two sigmoid searches 64 keys a round)
    const bool sm = u > kKeyNegInf && u <= kKeyPosInf;
    const float su = sm ? sigmoidf_tf(from_orderable(u)) : 0.f;
    const uint32_t lo = sm ? wave_lower_bound_sig(kKeyNegInf, u, su) : 0u;
    const uint32_t hi = sm ? wave_upper_bound_sig(u, kKeyPosInf, su) : 0u;
    if (t == 0) {
      s_above = 0;
      s_tie = 0;
      if (sm) {
        s_sig = su;
        s_sigmode = 1;
        s_win_lo = lo > kKeyNegInf + kWindowMargin ? lo - kWindowMargin : kKeyNegInf;
        s_tie_hi = hi;
      } else {
        s_sig = 0.f;
        s_sigmode = 0;
        s_win_lo = u;
        s_tie_hi = u;
      }
    }
  }
  __syncthreads();
  const uint32_t tie_hi = s_tie_hi, win_lo = s_win_lo;
  const float su = s_sig;
  const bool sigmode = s_sigmode != 0;
  const int room = kCap - k;  // tie slots after the k "above" slots
  auto is_tie = [&](uint32_t key, float v) {
    return key >= win_lo && key <= tie_hi && (sigmode ? sigmoidf_tf(v) == su : key == u);
  };
  wg_visit(p, len, [&](int i, float v) {
    const uint32_t key = orderable(v);
    const uint64_t e = ((uint64_t)__float_as_uint(v) << 32) | (uint32_t)i;
    const bool above = key > tie_hi;
    const int pa = wave_append(above, &s_above);
    if (pa >= 0 && pa < k) sk[pa] = e;
    const int pt = wave_append(!above && is_tie(key, v), &s_tie);
    if (pt >= 0 && pt < room) sk[k + pt] = e;
  });
  __syncthreads();
  const int G = min(s_above, k), T = s_tie;
  if (T <= room) {  // every tied key fits: shift them down behind the above keys
    for (int c0 = 0; c0 < T; c0 += kWG) {
      const int i = c0 + t;
      const uint64_t e = i < T ? sk[k + i] : 0ull;
      __syncthreads();
      if (i < T) sk[G + i] = e;
      __syncthreads();
    }
    return G + T;
  }
  // the tie group in index order until k: blocks of 4 keys per thread
  const int need = k - G;
  int found = 0;
  for (int b0 = 0; b0 < len && found < need; b0 += 4 * kWG) {
    const int i0 = b0 + 4 * t;
    bool hit[4];
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + j;
      hit[j] = false;
      if (i < len) {
        const float v = p[i];
        hit[j] = is_tie(orderable(v), v);
      }
      c += hit[j] ? 1u : 0u;
    }
    const uint32_t incl = wg_inclusive_scan(c, part);
    uint32_t pos = incl - c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (hit[j]) {
        if (found + (int)pos < need)
          sk[G + found + pos] = ((uint64_t)__float_as_uint(p[i0 + j]) << 32) | (uint32_t)(i0 + j);
        ++pos;
      }
    }
    if (t == kWG - 1) s_bin = (int)incl;  // block total
    __syncthreads();
    found += s_bin;
    __syncthreads();
  }
  return G + min(found, need);
}

// The k-th smallest (1-based) of the valid values, 8 per thread: a radix
// select relative to the smallest value, 4,096 bins of 2^sh keys a pass over
// [lo, lo + span): the candidates' sort keys share their top bits (sigmoids
// of one exponent or two), so bins taken from the top bits put thousands of
// LDS atomics on a few words; relative bins spread them, and a span under
// 2^24 (the usual case) needs two passes instead of three.
//
// cap > 0: stop at the first bin whose end leaves at most cap values at or
// below it (and at least k): any such bound serves the caller, which sorts
// the values at or below it (usually one pass instead of three).
__device__ uint32_t wg_kth_smallest(const uint32_t (&h)[8], const bool (&ok)[8], int k,
                                    uint32_t* hist, uint32_t* part, int cap = 0, bool dpp = false) {
  __shared__ int s_bin;
  __shared__ uint32_t s_lt, s_in;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t mn = 0xffffffffu, mx = 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (ok[j]) {
      mn = min(mn, h[j]);
      mx = max(mx, h[j]);
    }
  if (dpp) {  // (the lane permutations of bitonic1024_lanes)
    mn = min(mn, lane_xor32<32>(mn));
    mx = max(mx, lane_xor32<32>(mx));
    mn = min(mn, lane_xor32<16>(mn));
    mx = max(mx, lane_xor32<16>(mx));
    mn = min(mn, lane_xor32<8>(mn));
    mx = max(mx, lane_xor32<8>(mx));
    mn = min(mn, lane_xor32<4>(mn));
    mx = max(mx, lane_xor32<4>(mx));
    mn = min(mn, lane_xor32<2>(mn));
    mx = max(mx, lane_xor32<2>(mx));
    mn = min(mn, lane_xor32<1>(mn));
    mx = max(mx, lane_xor32<1>(mx));
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    }
  }
  if (lane == 0) {
    hist[w] = mn;
    hist[kWG / 64 + w] = mx;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kWG / 64; ++j) {
    mn = min(mn, hist[j]);
    mx = max(mx, hist[kWG / 64 + j]);
  }
  __syncthreads();
  uint32_t lo = mn;
  uint64_t span = (uint64_t)mx - mn + 1u;
  int krem = k;
  for (;;) {
    int sh = 0;
    while ((span + ((1ull << sh) - 1u)) >> sh > 4096u) ++sh;
    for (int i = t; i < 4096; i += kWG) hist[i] = 0;
    if (t == 0) {
      s_bin = 0;
      s_lt = 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (ok[j] && h[j] >= lo && (uint64_t)(h[j] - lo) < span)
        atomicAdd(&hist[(h[j] - lo) >> sh], 1u);
    __syncthreads();
    uint32_t c4[4], loc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c4[j] = hist[4 * t + j];
      loc += c4[j];
    }
    const uint32_t incl = wg_inclusive_scan(loc, part, dpp);
    const uint32_t before = incl - loc;
    if ((uint32_t)krem > before && (uint32_t)krem <= incl) {
      uint32_t acc = before;
      for (int j = 0; j < 4; ++j) {
        if ((uint32_t)krem <= acc + c4[j]) {
          s_bin = 4 * t + j;
          s_lt = acc;
          s_in = c4[j];
          break;
        }
        acc += c4[j];
      }
    }
    __syncthreads();
    const uint64_t off = (uint64_t)s_bin << sh;
    // (below: values under lo from earlier passes, k - krem of them)
    if (cap > 0 && (k - krem) + (int)(s_lt + s_in) <= cap)
      return (uint32_t)((uint64_t)lo + min<uint64_t>(off + (1ull << sh), span) - 1u);
    lo += (uint32_t)off;
    krem -= (int)s_lt;
    if (sh == 0) return lo;
    span = min<uint64_t>(span - off, 1ull << sh);
    __syncthreads();
  }
}

__global__ __launch_bounds__(kWG) void retina_finish_kernel(
    const float* __restrict__ base_a, const float* __restrict__ base_b, Levels lv, RetinaGeo g,
    int topk, float thresh, DeltaCfg dc, SegInfo* __restrict__ info,
    const int32_t* __restrict__ wcount, const uint64_t* __restrict__ wslot,
    const uint64_t* __restrict__ ovf, const uint64_t* __restrict__ cand,
    const int32_t* __restrict__ pcnt, int compact, float* __restrict__ cscore,
    float4* __restrict__ cbox, int32_t* __restrict__ ccls, int32_t* __restrict__ lvl_cnt,
    uint32_t* __restrict__ maxc, int32_t* __restrict__ err, int early, int lanes, int lanes_kth) {
  extern __shared__ uint64_t sk[];  // kCap entries
  __shared__ uint32_t hist[4096];
  __shared__ uint32_t part[kWG / 64];
  __shared__ int s_n, s_m, s_cnt, s_le;
  const uint64_t t_start = stamp(), c_start = cycles();
  const int s = blockIdx.x, n = s / g.L, l = s - n * g.L;
  const int t = threadIdx.x;
  const int xk = info[s].k, xexact = info[s].exact, xnovf = info[s].novf;
  const uint32_t xlo = info[s].exact_lo;
  if (xk == 0) {
    if (t == 0) lvl_cnt[s] = 0;
    return;
  }
  if (t == 0) {
    s_n = 0;
    s_m = 0;
    s_cnt = 0;
    s_le = 0;
  }
  __syncthreads();
  // gather the wave slots of the segment's chunks (order is irrelevant: sorted
  // below): every count in one round of loads, then the first two entries of
  // each hit slot in a second, further entries (rare) after
  const int cpi = g.chunk0[g.L];
  const int w0 = (n * cpi + g.chunk0[l]) * kCW;
  const int nw = (g.chunk0[l + 1] - g.chunk0[l]) * kCW;
  const size_t nslots = (size_t)g.N * cpi * kCW;
  bool ok = !xexact && xnovf <= kCap;
  int m = 0;
  auto put = [&](int p, uint64_t ent) {
    if (p < kCap) sk[p] = ent;
    m += orderable(__uint_as_float((uint32_t)(ent >> 32))) >= xlo ? 1 : 0;
  };
  if (ok) {
    // the overflow entries (collect's hits past a wave's 8 slots) are loaded
    // up front, alongside the first batch (their positions come later)
    constexpr int kOv = 1;  // (1,024 entries up front, the rest after the slots: registers)
    const uint64_t* osrc = ovf + (size_t)s * kCap;
    uint64_t ov[kOv];
#pragma unroll
    for (int j = 0; j < kOv; ++j) ov[j] = j * kWG + t < xnovf ? osrc[j * kWG + t] : 0ull;
    if (compact) {
      // the compacted parts: counts (one per part), their prefix by wave 0,
      // then every entry in one round of loads (<= kCap: 8 per thread)
      __shared__ int s_pre[65];
      const int np = g.part0[l + 1] - g.part0[l];
      const int gp0 = n * g.part0[g.L] + g.part0[l];
      if (t < 64) {
        int tot = 0;
        for (int p0 = 0; p0 < np; p0 += 64) {
          const int c = p0 + t < np ? pcnt[gp0 + p0 + t] : 0;
          int incl = c;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (t >= o) incl += y;
          }
          if (p0 + t < np && p0 + t < 64) s_pre[p0 + t] = tot + incl - c;
          tot += __shfl(incl, 63);
        }
        if (t == 0) {
          s_pre[min(np, 64)] = tot;
          s_n = tot;
        }
      }
      __syncthreads();
      const int tot = s_n;
      if (np <= 64 && tot + xnovf <= kCap) {
        uint64_t ent[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = j * kWG + t;
          ent[j] = 0ull;
          if (i < tot) {
            // the part holding entry i: the last p with s_pre[p] <= i (empty
            // parts repeat a prefix), by binary search -- six LDS rounds for
            // all eight entries together (the r6 linear walk was up to np
            // dependent rounds per entry)
            int p = 0;
#pragma unroll
            for (int step = 32; step > 0; step >>= 1)
              if (p + step < np && s_pre[p + step] <= i) p += step;
            ent[j] = cand[(size_t)(gp0 + p) * kPartCap + (i - s_pre[p])];
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j * kWG + t < tot) put(j * kWG + t, ent[j]);
      } else if (t == 0) {
        s_n = kCap + 1;  // (more parts than the prefix holds, or too many: the exact select)
      }
    }
    constexpr int U = 8;  // wave slots per thread per batch (1333x800 P3: 11,812 in two)
    for (int e0 = 0; e0 < (compact ? 0 : nw); e0 += U * kWG) {
      int cc[U], pos[U];
      uint64_t e1[U], e2[U];
      // the first two entries of every slot load with its count, unconditionally
      // (a slot's rows always exist; entries past its count are ignored)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + u * kWG + t;
        const uint64_t* src = wslot + (size_t)(w0 + min(e, nw - 1));
        cc[u] = e < nw ? min(wcount[w0 + e], kWaveSlots) : 0;
        e1[u] = src[0];
        e2[u] = src[nslots];
      }
      // positions: per wave one LDS atomic per batch row (wave prefix of the counts)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int incl = cc[u];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(incl, o);
          if ((t & 63) >= o) incl += y;
        }
        const int wtot = __shfl(incl, 63);
        int b = 0;
        if ((t & 63) == 63 && wtot) b = atomicAdd(&s_n, wtot);
        pos[u] = __shfl(b, 63) + incl - cc[u];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (cc[u] > 0) put(pos[u], e1[u]);
        if (cc[u] > 1) put(pos[u] + 1, e2[u]);
        for (int j = 2; j < cc[u]; ++j)
          put(pos[u] + j, wslot[(size_t)j * nslots + (w0 + e0 + u * kWG + t)]);
      }
    }
    __syncthreads();
    const int nreg = s_n;
#pragma unroll
    for (int j = 0; j < kOv; ++j) {
      const int i = j * kWG + t;
      if (i < xnovf && nreg + i < kCap) put(nreg + i, ov[j]);
    }
    for (int i = kOv * kWG + t; i < xnovf; i += kWG)
      if (nreg + i < kCap) put(nreg + i, osrc[i]);
    if (m) atomicAdd(&s_m, m);
  }
  __syncthreads();
  const int nreg = s_n;
  ok = ok && nreg + xnovf <= kCap;
  ok = ok && s_m >= xk;
  const uint64_t t_gather = stamp(), c_gather = cycles();
  int nc = nreg + xnovf;
  if (!ok) {
    __syncthreads();
    nc = exact_select(seg_ptr(base_a, lv, n, l, g.K), g.len[l], xk, sk, hist, part, err);
  }
  __syncthreads();
  const uint64_t t_cand = stamp(), c_cand = cycles();
  // sort keys (~orderable(sigmoid) << 32 | index), 8 per thread in registers
  uint64_t kv[8];
  uint32_t hi[8];
  bool valid[8];

#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int i = j * kWG + t;
    valid[j] = i < nc;
    kv[j] = ~0ull;
    if (valid[j]) {
      const uint64_t e = sk[i];
      const float sc = sigmoidf_tf(__uint_as_float((uint32_t)(e >> 32)));
      kv[j] = ((uint64_t)(~orderable(sc)) << 32) | (uint32_t)e;
    }
    hi[j] = (uint32_t)(kv[j] >> 32);
  }
  const int kk = min(xk, nc);
  __syncthreads();
  // the kk smallest keys: all keys whose score word is <= the kk-th smallest
  // one, when at most 1,024 (ties beyond that: the general sort)
  const uint64_t t_keys = stamp();
  const uint32_t thr32 = nc <= kWG ? 0xffffffffu
                                    : wg_kth_smallest(hi, valid, kk, hist, part, early ? kWG : 0,
                                                      lanes_kth != 0);
  const uint64_t t_kth = stamp();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int pos = wave_append(valid[j] && hi[j] <= thr32, &s_le);
    if (pos >= 0 && pos < kWG) sk[pos] = kv[j];
  }
  __syncthreads();
  const uint64_t t_app = stamp();
  const int nle = s_le;
  if (nle <= kWG) {
    const uint64_t v = t < nle ? sk[t] : ~0ull;
    __syncthreads();
    const uint64_t sv = lanes ? bitonic1024_lanes(v, sk + kWG) : bitonic1024(v, sk + kWG);
    sk[t] = sv;
  } else {  // more than 1,024 keys tie at the k-th score: bitonic over all of them
#pragma unroll
    for (int j = 0; j < 8; ++j) sk[j * kWG + t] = kv[j];
    int npad = 2;
    while (npad < nc) npad <<= 1;
    __syncthreads();
    for (int size = 2; size <= npad; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const int lg = 31 - __clz(stride);
        for (int i = t; i < (npad >> 1); i += kWG) {
          const int lo = ((i >> lg) << (lg + 1)) + (i & (stride - 1));
          const int hi2 = lo + stride;
          const uint64_t a = sk[lo], b = sk[hi2];
          const bool asc = (lo & size) == 0;
          if ((a > b) == asc) {
            sk[lo] = b;
            sk[hi2] = a;
          }
        }
        __syncthreads();
      }
    }
  }
  __syncthreads();
  const uint64_t t_sorted = stamp(), c_sorted = cycles();
  // top-k, threshold (a prefix: sorted by score), decode
  const int capimg = g.L * topk;
  const size_t o0 = (size_t)n * capimg + (size_t)l * topk;
  const float4* d4 = reinterpret_cast<const float4*>(base_b + lv.off_b[l]) + (size_t)n * lv.img_b[l];
  uint32_t mymax = 0;
  bool any = false;
  int kept = 0;
  for (int j = t; j < kk; j += kWG) {
    const uint64_t key = sk[j];
    const float score = from_orderable(~(uint32_t)(key >> 32));
    if (score > thresh) {
      const int id = (int)(uint32_t)key;
      const int aidx = id / g.K, cls = id - aidx * g.K;
      const int hw = aidx / lv.A, a = aidx - hw * lv.A;
      const float4 anc = anchor_at(lv, l, hw, a);
      const float4 b = apply_delta(anc, d4[aidx], dc.wy, dc.wx, dc.wh, dc.ww, dc.clamp);
      cscore[o0 + j] = score;
      cbox[o0 + j] = b;
      ccls[o0 + j] = cls;
      const uint32_t bm = orderable(fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w)));
      mymax = any ? max(mymax, bm) : bm;
      any = true;
      ++kept;
    }
  }
  // per-wave max, one atomic per wave with a kept box
  const int lane = t & 63;
  uint32_t wm = any ? mymax : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wm = max(wm, (uint32_t)__shfl_xor((int)wm, o));
  if (__ballot(any) != 0 && lane == 0) atomicMax(&maxc[n], wm);
  if (kept) atomicAdd(&s_cnt, kept);
  __syncthreads();
  if (t == 0) {
    lvl_cnt[s] = s_cnt;
    info[s].ts[2] = t_start;
    info[s].ts[3] = t_gather;
    info[s].ts[4] = t_cand;
    info[s].ts[5] = t_sorted;
    info[s].ts[6] = stamp();
    info[s].cyc[2] = c_start;
    info[s].cyc[3] = c_gather;
    info[s].cyc[4] = c_cand;
    info[s].cyc[5] = c_sorted;
    info[s].cyc[6] = cycles();
    info[s].sub[0] = t_keys;
    info[s].sub[1] = t_kth;
    info[s].sub[2] = t_app;
    info[s].sub[3] = nle;
  }
}

// -------------------------------------------------------------------- nms
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// Merge rank of the per-level sorted candidate lists of one image, many
// workgroups per image (one candidate per thread): position = own rank +
// earlier levels' scores >= s + later levels' scores > s (the concat
// position breaks ties).  ord[image][position] = level * topk + rank.
// The merged position of candidate r (r-th of the concatenated level counts)
// and its level * topk + rank, from the per-level sorted scores sc.
__device__ __forceinline__ void rank_of(int r, const float* sc, const int* cnt, const int* cum,
                                        int L, int topk, int& pos, int& val) {
  int l = 0;
  while (l + 1 < L && cum[l + 1] <= r) ++l;
  const int j = r - cum[l];
  const float sv = sc[l * topk + j];
  int lo[D2MI_MAX_LEVELS], hi[D2MI_MAX_LEVELS];
#pragma unroll
  for (int m = 0; m < D2MI_MAX_LEVELS; ++m) {
    lo[m] = 0;
    hi[m] = (m < L && m != l) ? cnt[m] : 0;
  }
  // every level's search advances each step: D2MI_MAX_LEVELS probes in flight
  for (int step = 0; step < 14; ++step) {
    float pv[D2MI_MAX_LEVELS];
#pragma unroll
    for (int m = 0; m < D2MI_MAX_LEVELS; ++m)
      pv[m] = m < L ? sc[m * topk + min((lo[m] + hi[m]) >> 1, topk - 1)] : 0.f;
#pragma unroll
    for (int m = 0; m < D2MI_MAX_LEVELS; ++m) {
      if (lo[m] < hi[m]) {
        const int mid = (lo[m] + hi[m]) >> 1;
        if (m < l ? pv[m] >= sv : pv[m] > sv) lo[m] = mid + 1;
        else hi[m] = mid;
      }
    }
  }
  pos = j;
#pragma unroll
  for (int m = 0; m < D2MI_MAX_LEVELS; ++m) pos += lo[m];
  val = l * topk + j;
}

// The same rank restricted to merged positions < cap (the NMS's windowed rank,
// retina_var 4096): every other level is searched only over its first cap
// entries (a count of cap already puts the candidate at or past cap), so
// ceil(log2(cap + 1)) rounds, and the rounds stay a loop: this runs once per
// call from a cold instruction cache, where unrolled code costs more than
// the loop (about 0.3-0.5 us per KB, profiles/r5_icache_probe.log).
__device__ __forceinline__ void rank_of_capped(int r, const float* sc, const int* cnt, const int* cum,
                                               int L, int topk, int cap, int& pos, int& val) {
  int l = 0;
  while (l + 1 < L && cum[l + 1] <= r) ++l;
  const int j = r - cum[l];
  const float sv = sc[l * topk + j];
  int lo[D2MI_MAX_LEVELS], hi[D2MI_MAX_LEVELS];
#pragma unroll
  for (int m = 0; m < D2MI_MAX_LEVELS; ++m) {
    lo[m] = 0;
    hi[m] = (m < L && m != l) ? min(cnt[m], cap) : 0;
  }
  const int rounds = 32 - __clz(cap);
#pragma unroll 1
  for (int step = 0; step < rounds; ++step) {
#pragma unroll
    for (int m = 0; m < D2MI_MAX_LEVELS; ++m) {
      if (lo[m] < hi[m]) {
        const int mid = (lo[m] + hi[m]) >> 1;
        const float pv = sc[m * topk + mid];
        if (m < l ? pv >= sv : pv > sv) lo[m] = mid + 1;
        else hi[m] = mid;
      }
    }
  }
  pos = j;
#pragma unroll
  for (int m = 0; m < D2MI_MAX_LEVELS; ++m) pos += lo[m];
  val = l * topk + j;
}

constexpr int kRankT = 256;
__global__ __launch_bounds__(kRankT) void retina_rank_kernel(
    RetinaGeo g, int topk, const float* __restrict__ cscore, const int32_t* __restrict__ lvl_cnt,
    uint16_t* __restrict__ ord, int rolled) {
  extern __shared__ float sc[];  // [capimg]
  __shared__ int cnt[D2MI_MAX_LEVELS], cum[D2MI_MAX_LEVELS + 1];
  const int n = blockIdx.y, t = threadIdx.x;
  const int L = g.L, capimg = L * topk;
  const size_t o0 = (size_t)n * capimg;
  if (t == 0) {
    int acc = 0;
    for (int l = 0; l < L; ++l) {
      cnt[l] = lvl_cnt[n * L + l];
      cum[l] = acc;
      acc += cnt[l];
    }
    cum[L] = acc;
  }
  {
    constexpr int U = 8 * kWG / kRankT / 4;  // float4 per thread: capimg <= 8 * kWG
    float4 v[U];
    const float4* src = reinterpret_cast<const float4*>(cscore + o0);  // capimg % 4 == 0
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q4 = u * kRankT + t;
      v[u] = 4 * q4 < capimg ? src[q4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q4 = u * kRankT + t;
      if (4 * q4 < capimg) reinterpret_cast<float4*>(sc)[q4] = v[u];
    }
  }
  __syncthreads();
  const int r = blockIdx.x * kRankT + t;
  if (r >= cum[L]) return;
  int pos, val;
  // (retina_var 32: the rounds as a loop, ceil(log2(topk + 1)) of them --
  // every list holds <= topk, so the cap changes no position)
  if (rolled) rank_of_capped(r, sc, cnt, cum, L, topk, topk, pos, val);
  else rank_of(r, sc, cnt, cum, L, topk, pos, val);
  ord[o0 + pos] = (uint16_t)val;
}

// Corner-normalised boxes with a positive-area intersection (the only case
// in which tf_iou can exceed a non-negative threshold).
__device__ __forceinline__ bool boxes_meet(float4 a, float4 b) {
  return fminf(a.z, b.z) > fmaxf(a.x, b.x) && fminf(a.w, b.w) > fmaxf(a.y, b.y);
}

// Greedy NMS of image n's merged candidates by one workgroup (dyn: the LDS
// the kernel below declares).
__device__ __forceinline__ void nms_image(int n, float4* dyn, RetinaGeo g, int topk, const float* cscore,
                          const float4* cbox, const int32_t* ccls, const int32_t* lvl_cnt,
                          const uint16_t* ord, const uint32_t* maxc, float thr, int max_det,
                          SegInfo* info, float4* __restrict__ ob, float* __restrict__ os,
                          int32_t* __restrict__ oc, uint8_t* __restrict__ ov, int inl_rank,
                          int fast_iou, int fp_resolve) {
  const uint64_t t_start = stamp(), c_start = cycles();
  const bool fast = fast_iou != 0 && thr >= 0.f;
  const bool fp = fp_resolve != 0;
  __shared__ uint64_t colpart[kWG];  // (fp) per wave, per lane: column bits of the wave's rows
  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const int L = g.L, capimg = L * topk;
  // LDS: kept (offset box, box, score, class) [max_det], the window's
  // (offset box, box, score, class) [kWG]
  float4* kept_obox = dyn;
  float4* kept_box = kept_obox + max_det;
  float4* wobox = kept_box + max_det;
  float4* wbox = wobox + kWG;
  float* kept_sc = reinterpret_cast<float*>(wbox + kWG);
  int32_t* kept_cl = reinterpret_cast<int32_t*>(kept_sc + max_det);
  float* wsc = reinterpret_cast<float*>(kept_cl + max_det);
  int32_t* wcl = reinterpret_cast<int32_t*>(wsc + kWG);
  // inl_rank: the merge rank of the level lists in this workgroup (no rank
  // launch): the image's scores and its order in LDS after the window arrays
  float* rsc = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(wcl + kWG) + 15) &
                                        ~(uintptr_t)15);  // (float4 stores; 16 B of slack)
  uint16_t* lord = reinterpret_cast<uint16_t*>(rsc + capimg);
  __shared__ uint64_t diag[kTile], wsup[kWG / 64];
  __shared__ int s_total, s_nk;
  __shared__ int rcnt[D2MI_MAX_LEVELS], rcum[D2MI_MAX_LEVELS + 1];
  const size_t o0 = (size_t)n * capimg;
  if (t == 0) {
    int acc = 0;
    for (int l = 0; l < L; ++l) {
      rcnt[l] = lvl_cnt[n * L + l];
      rcum[l] = acc;
      acc += rcnt[l];
    }
    rcum[L] = acc;
    s_total = acc;
    s_nk = 0;
  }
  if (inl_rank) {
    const float4* src = reinterpret_cast<const float4*>(cscore + o0);  // capimg % 4 == 0
    for (int q4 = t; 4 * q4 < capimg; q4 += kWG) reinterpret_cast<float4*>(rsc)[q4] = src[q4];
  }
  __syncthreads();
  if (inl_rank == 1) {
    for (int r = t; r < s_total; r += kWG) {
      int pos, val;
      rank_of(r, rsc, rcnt, rcum, L, topk, pos, val);
      lord[pos] = (uint16_t)val;
    }
    __syncthreads();
  }
  const uint64_t t_ranked = stamp(), c_ranked = cycles();
  const int total = s_total;
  const float off1 = from_orderable(maxc[n]) + 1.f;
  int nk = 0;
  uint64_t t_win = 0, t_tile1 = 0, t_a = 0, t_b = 0, t_c = 0;
  int ntiles = 0;
  // inl_rank 2 (retina_var 4096): windows of kRankWin candidates, each ranked
  // here just before it is used -- a candidate at position j of its level's
  // list has j candidates above it, so a window [w0, w0 + W) only holds
  // candidates with j < w0 + W; the NMS usually ends inside the first window
  const int wsize = inl_rank == 2 ? kRankWin : kWG;
  for (int w0 = 0; w0 < total && nk < max_det; w0 += wsize) {
    // window: the next wsize candidates in score order
    const int wn = min(wsize, total - w0);
    if (inl_rank == 2) {
      const int lim = w0 + wsize;  // list positions that can land in this window
      for (int idx = t; idx < L * lim; idx += kWG) {
        const int l = idx / lim, j = idx - l * lim;
        if (j < rcnt[l]) {
          int pos, val;
          rank_of_capped(rcum[l] + j, rsc, rcnt, rcum, L, topk, lim, pos, val);
          if (pos >= w0 && pos < lim) lord[pos - w0] = (uint16_t)val;
        }
      }
      __syncthreads();
    }
    if (t < wn) {
      const int q = inl_rank == 2 ? (int)lord[t] : inl_rank ? (int)lord[w0 + t] : (int)ord[o0 + w0 + t];
      const float4 c = cbox[o0 + q];
      const int cl = ccls[o0 + q];
      const float off = (float)cl * off1;
      const float4 ob4 = make_float4(c.x + off, c.y + off, c.z + off, c.w + off);
      // (fast: stored corner-normalised -- tf_iou normalises its inputs, so
      // its value on these is the same bits)
      wobox[t] = fast ? make_float4(fminf(ob4.x, ob4.z), fminf(ob4.y, ob4.w), fmaxf(ob4.x, ob4.z),
                                    fmaxf(ob4.y, ob4.w))
                      : ob4;
      wbox[t] = c;
      wsc[t] = cscore[o0 + q];
      wcl[t] = cl;
    }
    __syncthreads();
    if (w0 == 0) t_win = stamp();
    for (int t0 = 0; t0 < wn && nk < max_det; t0 += kTile) {
      ++ntiles;
      const int rem = wn - t0;
      const float4 cb = lane < rem ? wobox[t0 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
      bool sup = false;
      // (fast: the IoU only where the normalised boxes intersect -- elsewhere
      // it is 0 or NaN, never > thr >= 0 -- and per row only when some lane does)
      if (fast) {
        for (int i = w; i < nk; i += kWG / 64) {
          const float4 kb = kept_obox[i];
          if (!sup && boxes_meet(kb, cb)) sup = tf_iou(kb, cb) > thr;
        }
      } else {
        for (int i = w; i < nk; i += kWG / 64) sup = sup || (tf_iou(kept_obox[i], cb) > thr);
      }
      const uint64_t ws = __ballot(sup);
      if (lane == 0) wsup[w] = ws;
      constexpr int RPW = kTile / (kWG / 64);  // tile rows per wave
      uint64_t colp = 0;  // (fp: this lane's column bits of the wave's rows)
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int r = w * RPW + rr;
        const bool live = r < rem && lane > r && lane < rem;
        uint64_t d;
        bool p;
        if (fast) {
          const float4 rb = wobox[t0 + r];
          const bool meet = live && boxes_meet(rb, cb);
          p = __ballot(meet) ? (meet && tf_iou(rb, cb) > thr) : false;
        } else {
          p = live && tf_iou(wobox[t0 + r], cb) > thr;
        }
        d = __ballot(p);
        colp |= p ? (1ull << r) : 0ull;
        if (lane == 0) diag[r] = d;
      }
      if (fp) colpart[w * 64 + lane] = colp;
      if (ntiles == 1) t_a = stamp();
      __syncthreads();
      if (ntiles == 1) t_b = stamp();
      if (w == 0) {
        uint64_t removed = 0;
#pragma unroll
        for (int vv = 0; vv < kWG / 64; ++vv) removed |= wsup[vv];
        if (rem < 64) removed |= ~((1ull << rem) - 1ull);
        uint64_t keptm = 0;
        int k2 = nk;
        if (fp) {
          // (retina_var 2048) the kept set as the fixed point of a ballot
          // over the column words (nms.hip's r5 scan): lane c is row c, kept
          // iff alive and no kept row < c suppresses it; row c is final after
          // c + 1 rounds, and the greedy set is the only fixed point
          uint64_t colD = 0;
#pragma unroll
          for (int vv = 0; vv < kWG / 64; ++vv) colD |= colpart[vv * 64 + lane];
          const bool alive = !((removed >> lane) & 1ull);
          uint64_t K = __ballot(alive);
          for (int it = 0; it <= 64; ++it) {
            const uint64_t K2 = __ballot(alive && (colD & K) == 0ull);
            if (K2 == K) break;
            K = K2;
          }
          const int room = max_det - nk;
          if (__popcll(K) > room) {  // the greedy stops at max_det: its first room rows
            uint64_t kk2 = 0, rest = K;
            for (int q = 0; q < room; ++q) {
              const uint64_t low = rest & (~rest + 1ull);
              kk2 |= low;
              rest ^= low;
            }
            K = kk2;
          }
          keptm = K;
          k2 = nk + __popcll(K);
        } else {
          const uint64_t my_diag = diag[lane];
          for (int r = 0; r < kTile; ++r) {
            if (k2 >= max_det) break;
            if (!((removed >> r) & 1ull)) {
              keptm |= 1ull << r;
              ++k2;
              removed |= readlane64(my_diag, r);
            }
          }
        }
        if ((keptm >> lane) & 1ull) {
          const int pos = nk + __popcll(keptm & ((1ull << lane) - 1ull));
          kept_obox[pos] = wobox[t0 + lane];
          kept_box[pos] = wbox[t0 + lane];
          kept_sc[pos] = wsc[t0 + lane];
          kept_cl[pos] = wcl[t0 + lane];
        }
        if (lane == 0) s_nk = k2;
        if (ntiles == 1) t_c = stamp();
      }
      __syncthreads();
      nk = s_nk;
      if (ntiles == 1) t_tile1 = stamp();
    }
  }
  const uint64_t t_loop = stamp();
  for (int i = t; i < max_det; i += kWG) {
    const size_t o = (size_t)n * max_det + i;
    const bool k = i < nk;
    ob[o] = k ? kept_box[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    os[o] = k ? kept_sc[i] : 0.f;
    oc[o] = k ? kept_cl[i] : 0;
    ov[o] = k ? 1 : 0;
  }
  if (t == 0) {
    info[n * L].ts[7] = t_start;
    info[n * L].ts[8] = t_ranked;
    info[n * L].ts[9] = stamp();
    info[n * L].cyc[7] = c_start;
    info[n * L].cyc[8] = c_ranked;
    info[n * L].cyc[9] = cycles();
    info[n * L].sub[4] = t_win;
    info[n * L].sub[5] = ntiles;
    info[n * L].sub[6] = t_tile1;
    info[n * L].sub[7] = t_loop;
    if (L > 1) {  // (first tile: diag rows done, after the barrier, resolved)
      info[n * L + 1].sub[4] = t_a;
      info[n * L + 1].sub[5] = t_b;
      info[n * L + 1].sub[6] = t_c;
    }
  }
}

__global__ __launch_bounds__(kWG) void retina_nms_kernel(
    RetinaGeo g, int topk, const float* __restrict__ cscore, const float4* __restrict__ cbox,
    const int32_t* __restrict__ ccls, const int32_t* __restrict__ lvl_cnt,
    const uint16_t* __restrict__ ord, const uint32_t* __restrict__ maxc, float thr, int max_det,
    SegInfo* __restrict__ info, float4* __restrict__ ob, float* __restrict__ os,
    int32_t* __restrict__ oc, uint8_t* __restrict__ ov, int inl_rank, int fast_iou, int fp_resolve) {
  extern __shared__ float4 dyn[];
  nms_image(blockIdx.x, dyn, g, topk, cscore, cbox, ccls, lvl_cnt, ord, maxc, thr, max_det, info, ob,
            os, oc, ov, inl_rank, fast_iou, fp_resolve);
}

struct FusedWs {
  SegInfo* info;
  int32_t* wcount;
  uint64_t* wslot;
  uint64_t* ovf;
  float* cscore;
  float4* cbox;
  int32_t* ccls;
  int32_t* lvl_cnt;
  uint32_t* maxc;
  uint16_t* ord;
  uint64_t* cand;
  int32_t* pcnt;
};
template <typename WS>
void fused_layout(WS& w, FusedWs* o, int N, int L, int k, int chunks, int parts) {
  const int S = N * L;
  const size_t C = (size_t)N * L * k;
  auto a0 = w.template take<SegInfo>(S);
  auto a1 = w.template take<int32_t>((size_t)chunks * kCW);
  auto a2 = w.template take<uint64_t>((size_t)chunks * kCW * kWaveSlots);
  auto a3 = w.template take<uint64_t>((size_t)S * kCap);
  auto a4 = w.template take<float>(C);
  auto a5 = w.template take<float4>(C);
  auto a6 = w.template take<int32_t>(C);
  auto a7 = w.template take<int32_t>(S);
  auto a8 = w.template take<uint32_t>(N);
  auto a9 = w.template take<uint16_t>(C);
  auto a10 = w.template take<uint64_t>((size_t)parts * kPartCap);
  auto a11 = w.template take<int32_t>((size_t)parts);
  if (o)
    *o = FusedWs{(SegInfo*)a0, (int32_t*)a1, (uint64_t*)a2, (uint64_t*)a3, (float*)a4,
                 (float4*)a5, (int32_t*)a6, (int32_t*)a7, (uint32_t*)a8, (uint16_t*)a9,
                 (uint64_t*)a10, (int32_t*)a11};
}
struct SizerP {
  WorkspaceSizer z;
  template <typename T>
  T* take(size_t n) {
    z.take<T>(n);
    return nullptr;
  }
};

// per-level geometry; false when a level does not fit the int32 indexing
bool make_geo(RetinaGeo& g, const int32_t* level_hw, int L, int A, int K, int N) {
  g = RetinaGeo{};
  g.L = L;
  g.N = N;
  g.K = K;
  g.chunk0[0] = 0;
  g.part0[0] = 0;
  for (int l = 0; l < L; ++l) {
    const int64_t anchors = (int64_t)level_hw[2 * l] * level_hw[2 * l + 1] * A;
    const int64_t len = anchors * K;
    if (len >= (1ll << 31) - 8) return false;
    g.len[l] = (int32_t)len;
    g.anchors[l] = (int32_t)anchors;
    const int64_t c = g.chunk0[l] + (len + 3 + 4LL * kChunk4 - 1) / (4LL * kChunk4);
    if (c * N >= (1ll << 31) / kCW) return false;
    g.chunk0[l + 1] = (int32_t)c;
    g.part0[l + 1] = g.part0[l] + (int32_t)(((c - g.chunk0[l]) * kCW + kPT - 1) / kPT);
  }
  return true;
}
}  // namespace

bool retina_fused_eligible(int L, int k, int max_det) {
  return L >= 1 && L <= D2MI_MAX_LEVELS && k >= 1 && k <= kCap && (int64_t)L * k <= 8 * kWG &&
         (L * k) % 4 == 0 && max_det >= 1 && max_det <= 1000;
}

size_t retina_fused_workspace_size(int N, int L, const int32_t* level_hw, int A, int K, int k) {
  RetinaGeo g;
  if (!make_geo(g, level_hw, L, A, K, N)) return 0;
  SizerP s;
  fused_layout(s, nullptr, N, L, k, N * g.chunk0[L], N * g.part0[L]);
  return s.z.off;
}

int retinanet_fused(const float* const* cls, const float* const* box, const Levels& lv,
                    const int32_t* level_hw, int K, int N, int k, float score_thresh,
                    float nms_thresh, int max_det, DeltaCfg dc, float* out_boxes,
                    float* out_scores, int32_t* out_classes, uint8_t* out_valid, void* workspace,
                    size_t workspace_bytes, hipStream_t st, bool force_exact) {
  const int L = lv.L, S = N * L;
  D2MI_REQUIRE(retina_fused_eligible(L, k, max_det), "fused RetinaNet sizes out of range");
  // tuning "retina_var" (r6 bits; default 12018 = 2 + 16 + 32 + 64 + 128 +
  // 512 + 1024 + 2048 + 8192, 0 = the r5 form): 16 = the wave slots compacted by many workgroups before the
  // finish (one launch more), 64 = the finish's select stops at the first
  // bound that leaves <= 1,024 keys, 128 = the finish's bitonic exchanges in
  // DPP / permlane lane permutations, 512 = the finish's k-th select with
  // DPP / permlane reductions and scans, 1024 = the NMS's IoU only where
  // boxes intersect (exact), 2048 = the NMS tile resolved as a ballot fixed
  // point over column words, 4096 = no rank launch: the NMS ranks each
  // 128-candidate window itself, 8192 = the floor's ts-th maximum by a
  // radix select over the workgroup, 32 = the rank launch's search rounds
  // capped and kept as a loop, 2 = a small level's floor samples spread over
  // the whole level; 4 = floor and finish launched twice
  // (both idempotent: the stamps then time warm second launches)
  const int var = tuning(kTuneRetinaVar);
  RetinaGeo g;
  D2MI_REQUIRE(make_geo(g, level_hw, L, lv.A, K, N), "RetinaNet level too large");
  const int chunks = N * g.chunk0[L];
  Workspace w(workspace, workspace_bytes);
  FusedWs o;
  fused_layout(w, &o, N, L, k, chunks, N * g.part0[L]);
  D2MI_REQUIRE(w.ok(), "retinanet workspace too small (%zu < %zu)", workspace_bytes, w.off);
  const int reps = (var & 4) ? 2 : 1;
  for (int rep = 0; rep < reps; ++rep) {
    hipLaunchKernelGGL(retina_floor_kernel, dim3(S), dim3(kWG), 0, st, cls[0], lv, g, k,
                       force_exact ? 1 : 0, (var & 8192) ? 1 : 0, (var & 2) ? 1 : 0, o.info,
                       o.maxc);
    D2MI_LAUNCH_CHECK();
  }
  // persistent collect grid: the workgroups the device holds at once
  static int resident = 0;
  if (!resident) {
    int dev = 0, cus = 0, per = 0;
    D2MI_HIP(hipGetDevice(&dev));
    D2MI_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    D2MI_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, retina_collect_kernel, kCT, 0));
    resident = std::max(1, cus * std::max(1, per));
  }
  hipLaunchKernelGGL(retina_collect_kernel, dim3(std::min(chunks, resident)), dim3(kCT), 0, st, cls[0],
                     lv, g, o.info, o.wcount, o.wslot, o.ovf);
  D2MI_LAUNCH_CHECK();
  const int compact = (var & 16) ? 1 : 0;
  if (compact) {
    int maxp = 0;
    for (int l = 0; l < L; ++l) maxp = std::max(maxp, g.part0[l + 1] - g.part0[l]);
    hipLaunchKernelGGL(retina_compact_kernel, dim3(std::max(1, maxp), S), dim3(kPT), 0, st, g,
                       o.wcount, o.wslot, o.cand, o.pcnt);
    D2MI_LAUNCH_CHECK();
  }
  for (int rep = 0; rep < reps; ++rep) {
    hipLaunchKernelGGL(retina_finish_kernel, dim3(S), dim3(kWG), kCap * sizeof(uint64_t), st, cls[0],
                       box[0], lv, g, k, score_thresh, dc, o.info, o.wcount, o.wslot, o.ovf, o.cand,
                       o.pcnt, compact, o.cscore, o.cbox, o.ccls, o.lvl_cnt, o.maxc, error_word(),
                       (var & 64) ? 1 : 0, (var & 128) ? 1 : 0, (var & 512) ? 1 : 0);
    D2MI_LAUNCH_CHECK();
  }
  const int capimg = L * k;
  const int inl = tuning(kTuneRetinaRank) != 0 ? 1 : 0;
  // (tuning "retina_rank": 1 = the merge rank inside the NMS workgroup, 0 = its own launch;
  // measured: 165.6 vs 124.4 us per call -- one CU's LDS binary searches over ~4.7 k
  // candidates cost far more than the launch they save, profiles/r5_retina_post_ab_rank*.log)
  // (retina_var 4096: no rank launch -- the NMS ranks each 128-candidate
  // window itself, inl_rank 2)
  const int inl_arg = inl ? 1 : ((var & 4096) ? 2 : 0);
  if (!inl_arg) {
    hipLaunchKernelGGL(retina_rank_kernel, dim3((capimg + kRankT - 1) / kRankT, N), dim3(kRankT),
                       (size_t)capimg * sizeof(float), st, g, k, o.cscore, o.lvl_cnt, o.ord,
                       (var & 32) ? 1 : 0);
    D2MI_LAUNCH_CHECK();
  }
  const size_t lds = (size_t)(max_det + kWG) * (2 * sizeof(float4) + sizeof(float) + sizeof(int32_t)) +
                     (inl_arg ? 16 + (size_t)capimg * (sizeof(float) + sizeof(uint16_t)) : 0);
  hipLaunchKernelGGL(retina_nms_kernel, dim3(N), dim3(kWG), lds, st, g, k, o.cscore, o.cbox,
                     o.ccls, o.lvl_cnt, o.ord, o.maxc, nms_thresh, max_det, o.info,
                     reinterpret_cast<float4*>(out_boxes), out_scores, out_classes, out_valid, inl_arg,
                     (var & 1024) ? 1 : 0, (var & 2048) ? 1 : 0);
  D2MI_LAUNCH_CHECK();
  return 0;
}

}  // namespace d2mi
