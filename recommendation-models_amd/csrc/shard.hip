// shard.hip -- hash-sharded embedding table across ranks (one process per GPU), RCCL exchange.
//
// Replaces the reference's column-range-partitioned Angel PS matrices and their sparse pulls
// (ParRecModel.scala:74-105 ColumnRangePartitioner, pull :165-199, make* :279-306) for tables
// that are sharded over GPUs (BASELINE.json configs[3]: V = 100M over 8 x MI355X).
//
// Partitioning: owner(id) = p(id) mod N, local row = p(id) div N, a bijection [0, V) -> [N] x [ceil(V/N)].
// p = a keyed pseudo-random permutation of [0, V) (default key RMX_OWNER_HASH_DEFAULT, or
// rmx_shard_set_owner_hash): a 4-round Feistel network on the smallest even-width bit domain >= V,
// cycle-walked back into [0, V) -- strided or clustered real id spaces spread evenly over the owners,
// with no lookup table (BASELINE.json north_star: the table HASH-shards).  Key 0 = identity
// (owner = id mod N).
// One exchange step per batch on the caller's stream:
//   0. dedupe  : (rmx_shard_set_dedupe: off / on / auto, default auto) the batch's distinct ids, as
//                ParRecModel.distinctIntIndices (ParRecModel.scala:337-345) before the pull: an
//                open-addressing hash set in HBM (atomicCAS insert, linear probing) gives every
//                nnz its set slot; steps 1-5 then move one row per DISTINCT id and the final
//                perm[n] = slot of the distinct id of nnz n.
//   1. route   : per id, owner o and a slot in o's send bucket (block-local LDS histogram + one
//                global atomic per (block, owner) to reserve a range); send_ids[slot] = local row,
//                perm[n] = slot.  Copies only, so the bucket order inside a range is irrelevant.
//   2. counts  : grouped ncclSend/ncclRecv of one int per peer, then one D2H of the 2N counts
//                (the only host sync: NCCL needs host-side message sizes).
//   3. ids     : grouped send/recv of each bucket to its owner.
//   4. gather  : the owner copies emb[local][0..k) and w[local] for every received id.
//   5. rows    : grouped send/recv of the rows back, into the requester's bucket order.
//   (steps 3-5 skip this rank's own bucket: its rows are gathered straight into their slots)
//   6. forward : the model runs on (ids = perm, table = received rows): every kernel already
//                gathers through an id list, so nothing else changes and the outputs are bitwise
//                those of the replicated table (tests/test_shard.py).
// Steps 2, 3 and 5 go through a Transport: RCCL between processes (one rank per GPU, the product
// path), or an in-process exchange group (rmx_group: N virtual ranks, one host thread and one stream
// each, every grouped send/recv a device copy from the peer's posted buffer) that runs the SAME
// schedule -- offsets, own-bucket skip, buffer sizing -- at N > 1 on a single GPU.
// At one rank there is no exchange at all: route + the own-bucket gather, sized on the device (no
// host sync).
// A "loopback" shard (unique_id == NULL, no group) keeps all N partitions in this process on one
// GPU and serves every bucket in place: a single-thread check of the routing at N > 1.
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "rmx_models.hpp"

#define RMX_NCCL(expr)                                                                          \
  do {                                                                                          \
    ncclResult_t _r = (expr);                                                                   \
    if (_r != ncclSuccess) {                                                                    \
      ::rmx::set_error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " __FILE__ ":" + \
                       std::to_string(__LINE__) + ": " #expr);                                   \
      return RMX_E_COMM;                                                                        \
    }                                                                                           \
  } while (0)

namespace rmx {
// The exchange's grouped point-to-point ops (NCCL group semantics: every op between start() and
// end() is posted together; the k-th send from p to q pairs with the k-th recv of q from p).
struct Transport {
  virtual ~Transport() {}
  virtual int start() = 0;
  virtual int send(const void* p, size_t bytes, int peer, hipStream_t s) = 0;
  virtual int recv(void* p, size_t bytes, int peer, hipStream_t s) = 0;
  virtual int end(hipStream_t s) = 0;
};
}  // namespace rmx

// In-process exchange group: N virtual ranks (one host thread each) rendezvous in end().
struct rmx_group {
  int N = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;                      // a rank timed out: every later rendezvous fails
  struct Msg { const void* src; size_t bytes; };
  std::vector<std::vector<Msg>> posted;     // [from * N + to] sends of the current group
  std::vector<hipEvent_t> ev_send, ev_done; // per rank: its posted data ready / its copies done
  std::vector<int> attached;                // ranks with a shard
  int refs = 1;                             // the creator + one per attached shard
};

struct rmx_shard {
  rmx_ctx* ctx = nullptr;
  int64_t V = 0;
  int k = 0, N = 1, rank = 0;
  bool loopback = false;
  ncclComm_t comm = nullptr;
  // the communicator's life: 0 live, 1 aborted (rmx_shard_abort tore it down), 2 destroyed.  Abort and
  // destroy each claim it by compare-exchange from 0, so exactly one of ncclCommAbort / ncclCommDestroy
  // runs; the RCCL transport checks it before every call (nothing is posted on a torn-down comm)
  std::atomic<int> comm_state{0};
  rmx_group* group = nullptr;           // in-process exchange group (or null)
  std::unique_ptr<rmx::Transport> tr;   // RCCL or group transport (null: loopback)
  int64_t rows_per = 0;                 // ceil(V / N) local rows per partition
  uint64_t owner_key = RMX_OWNER_HASH_DEFAULT;  // Feistel key of p (set_owner_hash); 0: owner = id mod N
  bool filled = false;                  // rows written (the owner function is then fixed)
  int rs = 0;                           // row stride in floats: [emb k | w | pad], one 128-B line at k < 32
  std::vector<float*> part;             // partitions held here: [rows_per + 1][rs] (loopback: N); the
                                        // extra row stays zero (the row of an out-of-range id read in place)
  // per-batch buffers (grow only)
  int64_t cap_send = 0, cap_recv = 0;
  int64_t cap_slot[2] = {0, 0};         // ids each pull slot's perm holds (grown one slot at a time)
  int64_t cap_rows[2] = {0, 0};         // rows each pull slot's recv_emb / recv_w hold
  int64_t cap_sfix = 0;                 // send_ids elements (max(nnz, N * cap))
  int32_t* counts = nullptr;            // [4N]: send counts, recv counts, cursors, scratch
  int32_t* h_counts = nullptr;          // pinned host [2N]
  int32_t* send_ids = nullptr;          // [nnz] local rows, bucketed by owner
  int32_t* recv_ids = nullptr;          // [recv] local rows requested by the PEERS (own bucket excluded)
  float* send_emb = nullptr;            // [recv][k] rows gathered for them
  float* send_w = nullptr;              // [recv]
  // the exchange's output, the forward's input: two pull slots (rmx_shard_pull / rmx_forward_pulled
  // overlap batch i + 1's exchange with batch i's forward); perm / recv_* point at the active slot
  int32_t* perm = nullptr;              // [nnz] slot of id n
  float* recv_emb = nullptr;            // [nnz][k] rows for this rank's batch (bucket order)
  float* recv_w = nullptr;              // [nnz]
  int32_t* perm_s[2] = {nullptr, nullptr};
  float* recv_emb_s[2] = {nullptr, nullptr};
  float* recv_w_s[2] = {nullptr, nullptr};
  hipEvent_t ready[2] = {nullptr, nullptr};     // slot filled (recorded on the pull's stream)
  hipEvent_t consumed[2] = {nullptr, nullptr};  // slot read by its forward (on the forward's stream)
  bool consumed_rec[2] = {false, false};
  // one rank, no dedupe: the slot holds the batch's partition rows p(id) (perm_s), not copied rows --
  // the forward reads the [emb | w | pad] lines of the partition in place (no exchange, no row copy)
  bool slot_direct[2] = {false, false};
  int64_t slot_nnz[2] = {-1, -1};               // ids pulled into the slot, -1 = none pending
  // dedupe (step 0): 0 off, 1 on, 2 auto -- on for one batch, then off for the next kAutoSkip
  // batches when it removed under 10 % of the ids (uniform ids over a large V: the hash pass costs
  // more than the rows it saves), re-probed after them
  int dedupe = 2;
  int dedupe_skip = 0;
  int64_t cap_hash = 0;                 // hash-set slots (power of two >= 2 nnz)
  int32_t* hkeys = nullptr;             // [cap_hash] distinct ids (-1 = empty)
  int32_t* hvals = nullptr;             // [cap_hash] bucket slot of the distinct id
  int32_t* hslot = nullptr;             // [nnz] set slot of id n
  mutable int64_t last_sent = 0;        // ids sent by the last exchange (distinct ids when deduped)
  mutable bool last_sent_dev = false;   // one rank: last_sent is still on the device (counts[0])
  mutable int last_fixed = -1;          // >= 0: last_sent is the summary of that slot's fixed exchange (pinned)
  int32_t* bcnt = nullptr;              // [N][tiles] per-tile owner counts -> tile start offsets
  int64_t cap_tiles = 0;
  // Fixed-capacity exchange (N > 1 through a transport; knob "shard_fixed", default on): every peer bucket
  // has the host-known capacity cap (cap_of: ~1.1 nnz / N), so every message size is fixed and no count
  // has to reach the host before the rows move.  The first cap ids of bucket o go in send_ids[o][cap],
  // the rest (overflow) in send_ovf; each rank's header tells every peer its count and whether it
  // overflowed anywhere, so all ranks learn the same "any overflow" and agree on running a second,
  // counted round for the overflow ids (shard_resolve) -- never a different number of collectives.
  int64_t cap_fix = 0;                  // N * cap held by recv_fix / srow_*
  // The capacity must be the same on every rank (the message sizes pair up) without a host round trip,
  // so it comes from the PREVIOUS exchange: ~1.1 x the largest routed total of any rank there / N (every
  // rank reads the same maximum from its summary).  The first exchange has cap 0 (every id goes through
  // the counted overflow round) unless rmx_shard_set_batch_hint seeded it with the same value on every rank.
  int64_t cap_next = 0;
  int32_t* send_ovf = nullptr;          // [cap_send] overflow ids in bucket order
  int32_t* recv_fix = nullptr;          // [N][cap] ids requested by the peers
  float* srow_emb = nullptr;            // [N][cap][k] rows gathered for the peers
  float* srow_w = nullptr;              // [N][cap]
  int32_t* hdr = nullptr;               // device: headers sent [N][3] | received [N][3] | summary [2N + 2]
  int32_t* h_hdr_s[2] = {nullptr, nullptr};   // pinned per pull slot: the summary (counts sent, received, any, max total)
  hipEvent_t hdr_ev[2] = {nullptr, nullptr};  // the slot's summary has reached the host
  bool unresolved[2] = {false, false};  // a fixed exchange whose overflow check is pending
  hipStream_t slot_stream[2] = {nullptr, nullptr};  // its stream (the overflow round runs there)
  int64_t slot_cap[2] = {0, 0}, slot_n[2] = {0, 0};
  bool slot_dd[2] = {false, false};
  int64_t rounds2 = 0;                  // overflow rounds run so far
  int64_t cap_ovf = 0;                  // owner side of the overflow round (grown on demand)
  int32_t* recv_ovf = nullptr;
  float* ovf_emb = nullptr;
  float* ovf_w = nullptr;
  // the overflow round runs on its slot's stream (shard_resolve), which need not be the stream of the
  // ShardUse that called it (rmx_forward_pulled resolves outside one): the next exchange's stream waits
  // on this event before its route rewrites send_ovf / the row scratch
  hipEvent_t ovf_done = nullptr;
  bool ovf_pending = false;
  // RCCL calls between start() and end() of one grouped exchange hold this lock; rmx_shard_abort takes it
  // (bounded wait) before ncclCommAbort, so no ncclSend / ncclGroupEnd runs on a comm being torn down
  std::timed_mutex tr_mu;
  // an exchange failed on this rank after or before posting part of its ops: its peers' collectives no
  // longer pair up with this rank's, so every later exchange fails at once (abort and recreate the shard)
  bool failed = false;
  // one exchange at a time per shard; the per-batch buffers are ordered across streams like a
  // model's workspace (rmx::ModelUse)
  std::mutex mu;
  hipStream_t ws_stream = nullptr;
  hipEvent_t ws_fence = nullptr;
  bool ws_fence_lazy = false;  // (rmx::StreamUse)
};

namespace rmx {

namespace {

constexpr int kRouteThreads = 256, kRoutePer = 8, kRouteTile = kRouteThreads * kRoutePer, kMaxRanks = 64;

// Wave-aggregated bucket reservation: the lanes of a wave holding owner o (o >= 0) take
// consecutive ranks from one LDS atomic by the first such lane (one atomic per distinct owner in the
// wave instead of one per id: at N = 1 every id would hit the same LDS counter).
__device__ __forceinline__ int wave_reserve(int o, int* h) {
  const int lane = threadIdx.x & 63;
  uint64_t active = __ballot(o >= 0);
  int rank = 0;
  while (active) {
    const int leader = __ffsll((unsigned long long)active) - 1;
    const int lo = __shfl(o, leader);
    const uint64_t m = __ballot(o == lo);
    int base = 0;
    if (lane == leader) base = atomicAdd(&h[lo], __popcll(m));
    base = __shfl(base, leader);
    if (o == lo) rank = base + __popcll(m & ((1ull << lane) - 1));
    active &= ~m;
  }
  return rank;
}

// Routing = count -> scan -> scatter with no global atomics: block b histograms its tile of
// kRouteTile ids by owner into bcnt[o][b] (wave-aggregated LDS counters), one block per owner scans
// its column into the tile's start offset, and the scatter pass recomputes the in-tile ranks.
// The keyed permutation p of [0, V) (OwnerPerm.key == 0: identity): a 4-round Feistel network on
// the square domain Z_a x Z_a, a = ceil(sqrt(V)) (x = L a + R), each round (L, R) -> (R, (L + F_r(R))
// mod a) with F_r(R) = mulhi(fmix32(R ^ k_r), a) (the murmur3 finaliser; k_r four 32-bit round keys
// drawn from the key by splitmix64).  Cycle-walked back into [0, V): the domain exceeds V by < 2a,
// so a walk is rare (none at V = a^2, e.g. V = 10^8); every cycle re-enters [0, V) only if it started
// there.  All 32-bit integer work, ~40 instructions per id.
struct OwnerPerm {
  uint64_t key = 0;
  uint32_t a = 1;
  uint32_t rk[4] = {0, 0, 0, 0};
  int64_t V = 0;
};
__device__ __host__ __forceinline__ uint32_t owner_round(uint32_t x, uint32_t rk, uint32_t a) {
  uint32_t h = x ^ rk;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return (uint32_t)(((uint64_t)h * a) >> 32);  // uniform in [0, a)
}
__device__ __host__ __forceinline__ uint32_t feistel_once(uint32_t x, const OwnerPerm& op, bool inverse) {
  const uint32_t a = op.a;
  uint32_t L = x / a, R = x - L * a;
  if (!inverse) {
    for (int r = 0; r < 4; ++r) {
      const uint32_t t = owner_round(R, op.rk[r], a);
      const uint32_t s = L + t;
      L = R;
      R = s >= a ? s - a : s;
    }
  } else {
    for (int r = 3; r >= 0; --r) {
      const uint32_t t = owner_round(L, op.rk[r], a);
      const uint32_t l = R >= t ? R - t : R + a - t;
      R = L;
      L = l;
    }
  }
  return L * a + R;
}
__device__ __host__ __forceinline__ int64_t owner_perm(int64_t id, const OwnerPerm& op, bool inverse) {
  if (!op.key) return id;
  uint32_t y = feistel_once((uint32_t)id, op, inverse);
  while ((int64_t)y >= op.V) y = feistel_once(y, op, inverse);
  return y;
}

OwnerPerm owner_perm_of(uint64_t key, int64_t V) {
  OwnerPerm op;
  op.key = key;
  op.V = V;
  uint64_t a = (uint64_t)std::sqrt((double)std::max<int64_t>(V, 1));
  while ((int64_t)(a * a) < V) ++a;
  while (a > 1 && (int64_t)((a - 1) * (a - 1)) >= V) --a;
  op.a = (uint32_t)a;
  uint64_t z = key;
  for (int r = 0; r < 4; ++r) {  // round keys: splitmix64 of the key, successive states
    z += 0x9E3779B97F4A7C15ULL;
    uint64_t x = z;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    op.rk[r] = (uint32_t)(x ^ (x >> 31));
  }
  return op;
}
OwnerPerm owner_perm_of(const rmx_shard& sh) { return owner_perm_of(sh.owner_key, sh.V); }

__device__ __forceinline__ int route_owner(const int32_t* ids, int64_t n, int64_t nnz, int N, int* loc,
                                           const OwnerPerm& op) {
  if (n >= nnz) return -1;
  const int id = ids[n];
  // an empty hash-set slot (dedupe, -1), or an id outside [0, V): no owner.  (The cycle walk of the
  // keyed permutation ends only for ids inside [0, V): an id's cycle re-enters [0, V) only if it
  // started there.)
  if (id < 0 || id >= op.V) return -1;
  const int64_t p = owner_perm(id, op, false);
  *loc = (int)(p / N);
  return (int)(p % N);
}

__global__ __launch_bounds__(kRouteThreads) void route_count_kernel(int64_t nnz, int N, int nb,
                                                                   const int32_t* __restrict__ ids,
                                                                   int32_t* __restrict__ bcnt, OwnerPerm op) {
  __shared__ int h[kMaxRanks];
  for (int i = threadIdx.x; i < N; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRouteTile;
  int own[kRoutePer], loc;
#pragma unroll
  for (int u = 0; u < kRoutePer; ++u) own[u] = route_owner(ids, base + u * kRouteThreads + threadIdx.x, nnz, N, &loc, op);
#pragma unroll
  for (int u = 0; u < kRoutePer; ++u) (void)wave_reserve(own[u], h);
  __syncthreads();
  for (int o = threadIdx.x; o < N; o += blockDim.x) bcnt[(int64_t)o * nb + blockIdx.x] = h[o];
}

// block o: exclusive scan of bcnt[o][0..nb) in place; counts[o] = the column total
__global__ __launch_bounds__(1024) void route_scan_kernel(int nb, int32_t* __restrict__ bcnt,
                                                          int32_t* __restrict__ counts) {
  __shared__ int part[1024];
  int32_t* col = bcnt + (int64_t)blockIdx.x * nb;
  const int per = (nb + 1023) / 1024;
  const int t = threadIdx.x, i0 = t * per;
  int sum = 0;
  for (int i = i0; i < i0 + per && i < nb; ++i) sum += col[i];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan of the thread sums
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - sum;
  for (int i = i0; i < i0 + per && i < nb; ++i) {
    const int c = col[i];
    col[i] = run;
    run += c;
  }
  if (t == 1023) counts[blockIdx.x] = part[1023];
}

// Position of id n in its owner's bucket = tile start for o + rank in the tile.  Dense layout (cap < 0):
// slot = owner offset + position.  Fixed layout (cap >= 0): slot o * cap + position while position < cap,
// else the overflow list: send_ovf[q] with q = (overflow of the buckets before o) + position - cap, and
// the row slot N * cap + q.  An id with no owner (outside [0, V), or an empty dedupe slot) gets zslot,
// a row that stays zero.
__global__ __launch_bounds__(kRouteThreads) void route_scatter_kernel(int64_t nnz, int N, int nb,
                                                                     const int32_t* __restrict__ ids,
                                                                     const int32_t* __restrict__ counts,
                                                                     const int32_t* __restrict__ bstart,
                                                                     int32_t* __restrict__ send_ids,
                                                                     int32_t* __restrict__ perm, OwnerPerm op,
                                                                     int32_t cap, int32_t zslot,
                                                                     int32_t* __restrict__ send_ovf) {
  __shared__ int h[kMaxRanks], start[kMaxRanks], ovs[kMaxRanks];
  if (threadIdx.x == 0) {
    int s = 0, so = 0;
    for (int o = 0; o < N; ++o) {
      const int b = bstart[(int64_t)o * nb + blockIdx.x];
      start[o] = cap >= 0 ? b : s + b;  // fixed: the position inside the bucket
      ovs[o] = so;
      h[o] = 0;
      s += counts[o];
      so += cap >= 0 && counts[o] > cap ? counts[o] - cap : 0;
    }
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRouteTile;
  int own[kRoutePer], loc[kRoutePer];
#pragma unroll
  for (int u = 0; u < kRoutePer; ++u)
    own[u] = route_owner(ids, base + u * kRouteThreads + threadIdx.x, nnz, N, &loc[u], op);
#pragma unroll
  for (int u = 0; u < kRoutePer; ++u) {
    const int rk = wave_reserve(own[u], h);
    const int64_t n = base + u * kRouteThreads + threadIdx.x;
    if (own[u] >= 0) {
      const int pos = start[own[u]] + rk;
      if (cap < 0) {
        send_ids[pos] = loc[u];
        perm[n] = pos;
      } else if (pos < cap) {
        send_ids[own[u] * cap + pos] = loc[u];
        perm[n] = own[u] * cap + pos;
      } else {
        const int q = ovs[own[u]] + pos - cap;
        send_ovf[q] = loc[u];
        perm[n] = N * cap + q;
      }
    } else if (n < nnz) {
      perm[n] = zslot;  // no owner: the zero row
    }
  }
}

// rows for requested local ids out of a partition of [emb k | w | pad] rows (stride rs floats).
// k = 16, rs = 32: 8 lanes per row, one float4 each from the row's single 128-B line -- lanes 0-3
// the embedding, lane 4 the first-order weight (+ padding), lanes 5-7 idle -- so one id costs one
// memory line (a [V][k] table plus a separate [V] weight array costs two); generic otherwise.
// dcount (nullable): the row count lives on the device (the one-rank exchange, no host sync); n is
// then the grid's upper bound.
__global__ __launch_bounds__(256) void owner_gather_kernel(int64_t n, const int32_t* __restrict__ dcount, int k, int rs,
                                                          const int32_t* __restrict__ rows,
                                                          const float* __restrict__ part,
                                                          float* __restrict__ out_emb, float* __restrict__ out_w) {
  if (dcount) n = min(n, (int64_t)*dcount);
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k == 16 && rs == 32) {
    const int64_t i = t >> 3;
    const int c = (int)(t & 7);
    if (i >= n || c > 4) return;
    const int r = rows[i];
    const float4 v = reinterpret_cast<const float4*>(part)[(int64_t)r * 8 + c];
    if (c < 4)
      reinterpret_cast<float4*>(out_emb)[i * 4 + c] = v;
    else
      out_w[i] = v.x;
    return;
  }
  if (t >= n) return;
  const float* row = part + (int64_t)rows[t] * rs;
  for (int j = 0; j < k; ++j) out_emb[t * k + j] = row[j];
  out_w[t] = row[k];
}

// headers of the fixed exchange: to every peer o {count of bucket o, this rank overflowed anywhere,
// this rank's routed total}
__global__ void fixed_header_kernel(int N, int32_t cap, const int32_t* __restrict__ counts, int32_t* __restrict__ hdr) {
  int any = 0, tot = 0;
  for (int p = 0; p < N; ++p) {
    any |= counts[p] > cap ? 1 : 0;
    tot += counts[p];
  }
  for (int o = threadIdx.x; o < N; o += blockDim.x) {
    hdr[3 * o] = counts[o];
    hdr[3 * o + 1] = any;
    hdr[3 * o + 2] = tot;
  }
}

// the summary the host reads later: counts sent [N], counts received [N] (own bucket: its own count),
// the OR of every rank's overflow flag and the largest routed total of any rank -- the last two the
// same on every rank
__global__ void fixed_summary_kernel(int N, int me, const int32_t* __restrict__ counts, const int32_t* __restrict__ hs,
                                     const int32_t* __restrict__ hr, int32_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  int any = hs[3 * me + 1], mx = hs[3 * me + 2];
  for (int o = 0; o < N; ++o) {
    out[o] = counts[o];
    out[N + o] = o == me ? counts[me] : hr[3 * o];
    if (o != me) {
      any |= hr[3 * o + 1];
      mx = max(mx, hr[3 * o + 2]);
    }
  }
  out[2 * N] = any;
  out[2 * N + 1] = mx;
}

// Owner gather of the fixed exchange, one launch: for a peer o, row j < min(its count, cap) of its
// request recv_fix[o][j] into srow[o][j]; for the own bucket, send_ids[me][j] straight into this rank's
// received rows (slot me * cap + j).  Lane map as owner_gather_kernel (k = 16 line rows: 8 lanes).
__global__ __launch_bounds__(256) void fixed_gather_kernel(int N, int me, int32_t cap, int k, int rs,
                                                          const int32_t* __restrict__ counts,
                                                          const int32_t* __restrict__ hr,
                                                          const int32_t* __restrict__ send_ids,
                                                          const int32_t* __restrict__ recv_fix,
                                                          const float* __restrict__ part, float* __restrict__ srow_emb,
                                                          float* __restrict__ srow_w, float* __restrict__ recv_emb,
                                                          float* __restrict__ recv_w) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool fast = k == 16 && rs == 32;
  const int64_t i = fast ? t >> 3 : t;
  if (i >= (int64_t)N * cap) return;
  const int o = (int)(i / cap), j = (int)(i - (int64_t)o * cap);
  const int cnt = min(o == me ? counts[me] : hr[3 * o], cap);
  if (j >= cnt) return;
  const int r = o == me ? send_ids[i] : recv_fix[i];
  float* oe = o == me ? recv_emb : srow_emb;
  float* ow = o == me ? recv_w : srow_w;
  if (fast) {
    const int c = (int)(t & 7);
    if (c > 4) return;
    const float4 v = reinterpret_cast<const float4*>(part)[(int64_t)r * 8 + c];
    if (c < 4)
      reinterpret_cast<float4*>(oe)[i * 4 + c] = v;
    else
      ow[i] = v.x;
    return;
  }
  const float* row = part + (int64_t)r * rs;
  for (int q = 0; q < k; ++q) oe[i * k + q] = row[q];
  ow[i] = row[k];
}

// One rank, no dedupe: routing is the identity (every id is this rank's own, bucket order = batch
// order), so the count / scan / scatter passes are skipped and one pass gathers the rows in batch
// order: perm[n] = n, rows[n] = partition row p(ids[n]).  Same row layout and lane map as
// owner_gather_kernel; an id outside [0, V) gets a zero row (no read).
__global__ __launch_bounds__(256) void own_gather_kernel(int64_t n, int k, int rs, const int32_t* __restrict__ ids,
                                                        const float* __restrict__ part, float* __restrict__ out_emb,
                                                        float* __restrict__ out_w, int32_t* __restrict__ perm,
                                                        OwnerPerm op) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k == 16 && rs == 32) {
    const int64_t i = t >> 3;
    const int c = (int)(t & 7);
    if (i >= n || c > 5) return;
    if (c == 5) {
      perm[i] = (int32_t)i;
      return;
    }
    const int id = ids[i];
    const bool ok = id >= 0 && id < op.V;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) v = reinterpret_cast<const float4*>(part)[owner_perm(id, op, false) * 8 + c];
    if (c < 4)
      reinterpret_cast<float4*>(out_emb)[i * 4 + c] = v;
    else
      out_w[i] = v.x;
    return;
  }
  if (t >= n) return;
  const int id = ids[t];
  const bool ok = id >= 0 && id < op.V;
  const float* row = part + (ok ? owner_perm(id, op, false) : 0) * rs;
  for (int j = 0; j < k; ++j) out_emb[t * k + j] = ok ? row[j] : 0.f;
  out_w[t] = ok ? row[k] : 0.f;
  perm[t] = (int32_t)t;
}

__global__ __launch_bounds__(256) void iota_kernel(int64_t n, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)i;
}

// One rank, read in place: rows[n] = p(ids[n]), the partition row of id n (an id outside [0, V)
// gets the zero row `zrow`).  The forward then gathers the [emb | w | pad] lines straight from the
// partition: no route, no row copy.
__global__ __launch_bounds__(256) void own_rows_kernel(int64_t n, const int32_t* __restrict__ ids, int32_t zrow,
                                                      int32_t* __restrict__ rows, OwnerPerm op) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int id = ids[i];
  rows[i] = (id >= 0 && id < op.V) ? (int32_t)owner_perm(id, op, false) : zrow;
}

// step 0: insert ids[n] into the hash set; hslot[n] = its slot (first inserter claims an empty one)
__global__ __launch_bounds__(256) void dedupe_insert_kernel(int64_t nnz, const int32_t* __restrict__ ids,
                                                           uint32_t mask, int shift, int32_t* __restrict__ keys,
                                                           int32_t* __restrict__ hslot) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= nnz) return;
  const int32_t id = ids[n];
  // Fibonacci hashing: the TOP bits of the 64-bit product (the low bits of id * odd depend only on
  // the low bits of id, which clusters field-structured ids into long probe chains)
  uint32_t h = (uint32_t)(((uint64_t)(uint32_t)id * 0x9E3779B97F4A7C15ull) >> shift);
  while (true) {
    // a slot changes only once (-1 -> id): a plain read that already shows an id is final, so
    // repeated ids (skewed batches) mostly skip the device-scope atomic
    const int32_t seen = __builtin_nontemporal_load(&keys[h]);
    if (seen == id) break;
    if (seen == -1) {
      const int32_t old = atomicCAS(&keys[h], -1, id);
      if (old == -1 || old == id) break;
    }
    h = (h + 1) & mask;  // load factor <= 1/2: terminates
  }
  hslot[n] = (int32_t)h;
}

// perm[n] = bucket slot of the distinct id of nnz n
__global__ __launch_bounds__(256) void dedupe_perm_kernel(int64_t nnz, const int32_t* __restrict__ hslot,
                                                         const int32_t* __restrict__ hvals,
                                                         int32_t* __restrict__ perm) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n < nnz) perm[n] = hvals[hslot[n]];
}

__device__ __forceinline__ uint64_t splitmix64_d(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

// owned rows of partition `part`: global id = l*N + part, values of the global generator
// (oracle orc_gen_table / fill_table_kernel): bit-identical to the replicated table's rows
__global__ void shard_fill_kernel(uint64_t seed, int64_t V, int64_t rows_per, int N, int part, int k, int rs,
                                  float scale, float* __restrict__ rowsbuf, OwnerPerm op) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows_per * rs) return;
  const int64_t l = i / rs;
  const int j = (int)(i - l * rs);
  const int64_t pid = l * N + part;                              // position in p's image
  const int64_t id = pid < V ? owner_perm(pid, op, true) : V;    // the global id stored there
  float v = 0.f;
  if (id < V && j <= k) {  // j == k: the first-order weight; j > k: padding
    const uint64_t h = splitmix64_d(seed ^ (uint64_t)(id * (k + 1) + j));
    v = (float)((int32_t)(h >> 40) - 8388608) * scale;
  }
  rowsbuf[i] = v;
}

}  // namespace

namespace {

template <class T>
int realloc_dev(T** p, int64_t n) {
  if (*p) RMX_HIP(hipFree(*p));
  *p = nullptr;
  if (hipMalloc((void**)p, sizeof(T) * std::max<int64_t>(n, 1)) != hipSuccess) {
    set_error("shard: out of device memory (" + std::to_string(n * (int64_t)sizeof(T)) + " bytes)");
    return RMX_E_NOMEM;
  }
  return RMX_OK;
}

// [nnz]-sized buffers of this rank's batch: the exchange's scratch, and pull slot `slot` only.
// The other slot may hold a pull its forward has not consumed (or is still reading): it is never
// touched here.  The slot being grown has no pending pull (rmx_shard_pull refuses one), and the
// device sync retires any forward still reading its old buffers.  nfix: N * cap of a fixed exchange
// (0: dense buckets) -- send_ids then holds [N][cap] and the slot's rows nfix + nnz + 1 (the fixed
// buckets, the overflow rows, the zero row).
int ensure_batch(rmx_shard& sh, int64_t nnz, int slot, int64_t nfix = 0) {
  const int64_t nrows = nfix + nnz + 1;
  if (nnz <= sh.cap_send && nfix <= sh.cap_sfix && nnz <= sh.cap_slot[slot] && nrows <= sh.cap_rows[slot])
    return RMX_OK;
  RMX_HIP(hipDeviceSynchronize());  // in-flight work on any stream may still use the old buffers
  int st;
  if (nnz > sh.cap_send || nfix > sh.cap_sfix) {
    const int64_t n = std::max(nnz, sh.cap_send);
    int64_t hc = 1024;
    while (hc < 2 * n) hc <<= 1;
    const int64_t sf = std::max(std::max(n, nfix), sh.cap_sfix);
    if ((st = realloc_dev(&sh.send_ids, sf)) || (st = realloc_dev(&sh.send_ovf, n)) ||
        (st = realloc_dev(&sh.hslot, n)) || (st = realloc_dev(&sh.hkeys, hc)) || (st = realloc_dev(&sh.hvals, hc))) {
      sh.cap_send = sh.cap_hash = sh.cap_sfix = 0;
      return st;
    }
    sh.cap_send = n;
    sh.cap_sfix = sf;
    sh.cap_hash = hc;
  }
  if (nnz > sh.cap_slot[slot] || nrows > sh.cap_rows[slot]) {
    const int64_t n = std::max(nnz, sh.cap_slot[slot]), r = std::max(nrows, sh.cap_rows[slot]);
    if ((st = realloc_dev(&sh.perm_s[slot], n)) || (st = realloc_dev(&sh.recv_emb_s[slot], r * sh.k)) ||
        (st = realloc_dev(&sh.recv_w_s[slot], r))) {
      sh.cap_slot[slot] = sh.cap_rows[slot] = 0;
      return st;
    }
    sh.cap_slot[slot] = n;
    sh.cap_rows[slot] = r;
  }
  return RMX_OK;
}

// [N * cap]-sized owner-side buffers of the fixed exchange
int ensure_fixed(rmx_shard& sh, int64_t nfix) {
  if (nfix <= sh.cap_fix) return RMX_OK;
  RMX_HIP(hipDeviceSynchronize());  // a peer's copy of the old rows may still be in flight
  int st;
  if ((st = realloc_dev(&sh.recv_fix, nfix)) || (st = realloc_dev(&sh.srow_emb, nfix * sh.k)) ||
      (st = realloc_dev(&sh.srow_w, nfix))) {
    sh.cap_fix = 0;
    return st;
  }
  sh.cap_fix = nfix;
  return RMX_OK;
}

// owner side of the overflow round
int ensure_ovf(rmx_shard& sh, int64_t n) {
  if (n <= sh.cap_ovf) return RMX_OK;
  RMX_HIP(hipDeviceSynchronize());
  int st;
  if ((st = realloc_dev(&sh.recv_ovf, n)) || (st = realloc_dev(&sh.ovf_emb, n * sh.k)) ||
      (st = realloc_dev(&sh.ovf_w, n))) {
    sh.cap_ovf = 0;
    return st;
  }
  sh.cap_ovf = n;
  return RMX_OK;
}

// [N][tiles] routing scratch
int ensure_tiles(rmx_shard& sh, int64_t tiles) {
  if (tiles <= sh.cap_tiles) return RMX_OK;
  RMX_HIP(hipDeviceSynchronize());
  int st;
  if ((st = realloc_dev(&sh.bcnt, tiles * sh.N))) return st;
  sh.cap_tiles = tiles;
  return RMX_OK;
}

// [received]-sized buffers of the owner side
int ensure_recv(rmx_shard& sh, int64_t n) {
  if (n <= sh.cap_recv) return RMX_OK;
  int st;
  RMX_HIP(hipDeviceSynchronize());  // a peer's copy of the old rows may still be in flight
  if ((st = realloc_dev(&sh.recv_ids, n)) || (st = realloc_dev(&sh.send_emb, n * sh.k)) ||
      (st = realloc_dev(&sh.send_w, n))) {
    sh.cap_recv = 0;
    return st;
  }
  sh.cap_recv = n;
  return RMX_OK;
}

// the shard's lock + cross-stream order of its per-batch buffers (see rmx::StreamUse)
typedef StreamUse<rmx_shard> ShardUse;

int launch_owner_gather(hipStream_t s, int64_t n, int k, int rs, const int32_t* rows, const float* part,
                        float* out_emb, float* out_w, const int32_t* dcount = nullptr) {
  if (n <= 0) return RMX_OK;
  const int64_t threads = (k == 16 && rs == 32) ? n * 8 : n;
  hipLaunchKernelGGL(owner_gather_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, n, dcount, k, rs,
                     rows, part, out_emb, out_w);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// the un-permute of rmx_shard_gather: d_emb[i] = recv_emb[perm[i]] (dense [nnz][k] rows + weights)
__global__ __launch_bounds__(256) void unpermute_kernel(int64_t n, int k, const int32_t* __restrict__ perm,
                                                       const float* __restrict__ emb, const float* __restrict__ w,
                                                       float* __restrict__ out_emb, float* __restrict__ out_w) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k == 16) {  // 4 lanes per row, one float4 each
    const int64_t i = t >> 2;
    const int c = (int)(t & 3);
    if (i >= n) return;
    const int64_t r = perm[i];
    reinterpret_cast<float4*>(out_emb)[i * 4 + c] = reinterpret_cast<const float4*>(emb)[r * 4 + c];
    if (c == 0) out_w[i] = w[r];
    return;
  }
  if (t >= n) return;
  const int64_t r = perm[t];
  for (int j = 0; j < k; ++j) out_emb[t * k + j] = emb[r * k + j];
  out_w[t] = w[r];
}

}  // namespace

// ---------------------------------------------------------------- transports --
namespace {

// Every call first checks the shard's communicator state: after rmx_shard_abort (or during destroy)
// nothing more is posted on the torn-down communicator -- the exchange fails with RMX_E_COMM instead
// (an abort while the exchange was in flight used to reach ncclSend on a freed comm)
//  The check alone was check-then-act: an abort could free the comm between the check and
// the call.  start() now takes the shard's transport lock and end() releases it, so the whole bracket --
// check, posts, ncclGroupEnd -- runs with rmx_shard_abort held off; abort waits for the lock (bounded:
// a host thread stuck inside an RCCL call is exactly what abort is for, RCCL's abort may then run beside it).
// Every exchange passes start() and end() in pairs (also after a local error), so the lock is balanced.
struct RcclTransport : Transport {
  ncclComm_t comm;
  const std::atomic<int>* state;
  std::timed_mutex* mu;
  bool held = false;
  bool group_open = false;  // ncclGroupStart succeeded and its ncclGroupEnd has not run yet
  RcclTransport(ncclComm_t c, const std::atomic<int>* st, std::timed_mutex* m) : comm(c), state(st), mu(m) {}
  ~RcclTransport() override {
    if (held) mu->unlock();
  }
  int live() const {
    if (state->load() == 0) return RMX_OK;
    set_error("shard exchange: the communicator was aborted (rmx_shard_abort)");
    return RMX_E_COMM;
  }
  int start() override {
    if (!held) {
      mu->lock();
      held = true;
    }
    if (int e = live()) return e;
    RMX_NCCL(ncclGroupStart());
    group_open = true;
    return RMX_OK;
  }
  int send(const void* p, size_t bytes, int peer, hipStream_t s) override {
    if (int e = live()) return e;
    RMX_NCCL(ncclSend(p, bytes, ncclInt8, peer, comm, s));
    return RMX_OK;
  }
  int recv(void* p, size_t bytes, int peer, hipStream_t s) override {
    if (int e = live()) return e;
    RMX_NCCL(ncclRecv(p, bytes, ncclInt8, peer, comm, s));
    return RMX_OK;
  }
  int end(hipStream_t) override {
    struct Release {  // the bracket's lock, on every return
      RcclTransport* t;
      ~Release() {
        if (t->held) {
          t->held = false;
          t->mu->unlock();
        }
      }
    } rel{this};
    // A group that start() opened is closed here whatever happened in between: with the lock
    // held an abort normally waits, but rmx_shard_abort gives up waiting after 5 s and aborts the
    // communicator anyway, and this thread must not stay inside an open RCCL group -- a later shard's
    // ncclCommInitRank on it would run inside the leaked group.  On an aborted communicator the group's
    // own ncclGroupEnd result is ignored; the exchange reports RMX_E_COMM.
    const bool aborted = state->load() != 0;
    if (group_open) {
      group_open = false;
      const ncclResult_t r = ncclGroupEnd();
      if (!aborted && r != ncclSuccess) {
        set_error(std::string("RCCL ncclGroupEnd: ") + ncclGetErrorString(r));
        return RMX_E_COMM;
      }
    }
    if (aborted) {
      set_error("shard exchange: the communicator was aborted (rmx_shard_abort)");
      return RMX_E_COMM;
    }
    return RMX_OK;
  }
};

// Host rendezvous of the group's N threads; fails (and breaks the group) after kGroupTimeout.
constexpr auto kGroupTimeout = std::chrono::seconds(120);

int group_barrier(rmx_group& g) {
  std::unique_lock<std::mutex> lk(g.mu);
  if (g.broken) {
    set_error("exchange group: a rank failed to arrive earlier; the group is unusable");
    return RMX_E_COMM;
  }
  const uint64_t my = g.gen;
  if (++g.arrived == g.N) {
    g.arrived = 0;
    ++g.gen;
    g.cv.notify_all();
    return RMX_OK;
  }
  if (!g.cv.wait_for(lk, kGroupTimeout, [&] { return g.gen != my || g.broken; }) || g.broken) {
    g.broken = true;
    g.cv.notify_all();
    set_error("exchange group: peers did not reach the exchange (every rank must call it)");
    return RMX_E_COMM;
  }
  return RMX_OK;
}

// Every recv is a device copy from the matching send's buffer on the receiver's stream:
//   1. record ev_send[me] (this rank's posted data is ready), post the sends, rendezvous;
//   2. per recv: wait for ev_send[peer], copy; record ev_done[me] (my reads are done), rendezvous;
//   3. wait for ev_done[peer] of every peer I sent to, so later writes to my send buffers are safe.
// ev_send[p] / ev_done[p] are re-recorded only after a rendezvous that every reader has passed.
struct LocalTransport : Transport {
  rmx_group* g;
  int me;
  struct Op { void* p; size_t bytes; int peer; };
  std::vector<Op> sends, recvs;
  LocalTransport(rmx_group* gg, int r) : g(gg), me(r) {}
  int start() override {
    sends.clear();
    recvs.clear();
    return RMX_OK;
  }
  int send(const void* p, size_t bytes, int peer, hipStream_t) override {
    sends.push_back({const_cast<void*>(p), bytes, peer});
    return RMX_OK;
  }
  int recv(void* p, size_t bytes, int peer, hipStream_t) override {
    recvs.push_back({p, bytes, peer});
    return RMX_OK;
  }
  int end(hipStream_t s) override {
    const int N = g->N;
    // a failing HIP call must not skip the rendezvous (the peers would wait for this rank)
    int err = RMX_OK;
    auto hip = [&](hipError_t e, const char* what) {
      if (e != hipSuccess && err == RMX_OK) {
        set_error(std::string("exchange group: ") + what + ": " + hipGetErrorString(e));
        err = RMX_E_HIP;
      }
    };
    hip(hipEventRecord(g->ev_send[me], s), "hipEventRecord");
    {
      std::lock_guard<std::mutex> lk(g->mu);
      for (int to = 0; to < N; ++to) g->posted[(size_t)me * N + to].clear();
      for (const Op& o : sends) g->posted[(size_t)me * N + o.peer].push_back({o.p, o.bytes});
    }
    int st = group_barrier(*g);
    if (st) return st;
    std::vector<size_t> nth(N, 0);
    std::vector<char> waited(N, 0);
    for (const Op& o : recvs) {
      const auto& lst = g->posted[(size_t)o.peer * N + me];
      if (nth[o.peer] >= lst.size() || lst[nth[o.peer]].bytes != o.bytes) {
        if (err == RMX_OK) {
          set_error("exchange group: rank " + std::to_string(me) + " receives " + std::to_string(o.bytes) +
                    " bytes from rank " + std::to_string(o.peer) + " that posted no matching send");
          err = RMX_E_COMM;
        }
        continue;
      }
      if (!waited[o.peer]) {
        hip(hipStreamWaitEvent(s, g->ev_send[o.peer], 0), "hipStreamWaitEvent");
        waited[o.peer] = 1;
      }
      hip(hipMemcpyAsync(o.p, lst[nth[o.peer]].src, o.bytes, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync");
      ++nth[o.peer];
    }
    hip(hipEventRecord(g->ev_done[me], s), "hipEventRecord");
    if ((st = group_barrier(*g))) return st;
    std::vector<char> sent(N, 0);
    for (const Op& o : sends) sent[o.peer] = 1;
    for (int p = 0; p < N; ++p)
      if (sent[p]) hip(hipStreamWaitEvent(s, g->ev_done[p], 0), "hipStreamWaitEvent");
    return err;
  }
};

void group_unref(rmx_group* g) {
  bool last;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    last = --g->refs == 0;
  }
  if (!last) return;
  for (hipEvent_t e : g->ev_send)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : g->ev_done)
    if (e) (void)hipEventDestroy(e);
  delete g;
}

}  // namespace

int shard_create(rmx_ctx* ctx, int64_t V, int k, int N, int rank, const void* unique_id, rmx_group* group,
                 rmx_shard** out) {
  if (N < 1 || N > kMaxRanks || rank < 0 || rank >= N || V < N || k <= 0) {
    set_error("rmx_shard_create: bad arguments (need 1 <= nranks <= 64, 0 <= rank < nranks, rows >= nranks)");
    return RMX_E_INVALID;
  }
  if (V >= (int64_t(1) << 31)) {
    set_error("rmx_shard_create: rows must fit int32 (ParRecModel.scala:282 .toInt)");
    return RMX_E_INVALID;
  }
  if (group) {
    std::lock_guard<std::mutex> lk(group->mu);
    if (group->N != N) {
      set_error("rmx_shard_create_group: nranks differs from the group's size");
      return RMX_E_INVALID;
    }
    if (group->attached[rank]) {
      set_error("rmx_shard_create_group: rank " + std::to_string(rank) + " of the group already has a shard");
      return RMX_E_INVALID;
    }
  }
  RMX_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<rmx_shard> sh(new rmx_shard());
  sh->ctx = ctx;
  sh->V = V;
  sh->k = k;
  sh->N = N;
  sh->rank = rank;
  sh->loopback = unique_id == nullptr && group == nullptr;
  sh->rows_per = (V + N - 1) / N;
  sh->rs = (k + 1 + 31) / 32 * 32;  // [emb | w | pad]: a 128-B line per row for k < 32
  const int parts = sh->loopback ? N : 1;
  for (int p = 0; p < parts; ++p) {
    float* r = nullptr;
    if (hipMalloc(&r, sizeof(float) * (sh->rows_per + 1) * sh->rs) != hipSuccess) {
      for (float* q : sh->part) (void)hipFree(q);
      set_error("rmx_shard_create: out of device memory for the partition");
      return RMX_E_NOMEM;
    }
    sh->part.push_back(r);
  }
  RMX_HIP(hipMalloc(&sh->counts, sizeof(int32_t) * 4 * N));
  RMX_HIP(hipHostMalloc(&sh->h_counts, sizeof(int32_t) * 2 * N));
  RMX_HIP(hipMalloc(&sh->hdr, sizeof(int32_t) * (8 * N + 2)));
  for (int q = 0; q < 2; ++q) {
    RMX_HIP(hipHostMalloc(&sh->h_hdr_s[q], sizeof(int32_t) * (2 * N + 2)));
    RMX_HIP(hipEventCreateWithFlags(&sh->hdr_ev[q], hipEventDisableTiming));
  }
  if (group) {
    std::lock_guard<std::mutex> lk(group->mu);
    if (!group->ev_send[rank]) {
      RMX_HIP(hipEventCreateWithFlags(&group->ev_send[rank], hipEventDisableTiming));
      RMX_HIP(hipEventCreateWithFlags(&group->ev_done[rank], hipEventDisableTiming));
    }
    group->attached[rank] = 1;
    ++group->refs;
    sh->group = group;
    sh->tr.reset(new LocalTransport(group, rank));
  } else if (!sh->loopback) {
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    RMX_NCCL(ncclCommInitRank(&sh->comm, N, id, rank));
    sh->tr.reset(new RcclTransport(sh->comm, &sh->comm_state, &sh->tr_mu));
  }
  *out = sh.release();
  return RMX_OK;
}

int shard_destroy(rmx_shard* sh) {
  if (!sh) return RMX_OK;
  (void)hipSetDevice(sh->ctx->device);
  (void)hipDeviceSynchronize();  // the exchange may have run on any stream
  sh->tr.reset();
  if (sh->ws_fence) (void)hipEventDestroy(sh->ws_fence);
  if (sh->ovf_done) (void)hipEventDestroy(sh->ovf_done);
  int live = 0;  // claim the communicator: a concurrent rmx_shard_abort that got there first freed it
  if (sh->comm && sh->comm_state.compare_exchange_strong(live, 2)) ncclCommDestroy(sh->comm);
  if (sh->group) {
    {
      std::lock_guard<std::mutex> lk(sh->group->mu);
      sh->group->attached[sh->rank] = 0;
    }
    group_unref(sh->group);
  }
  for (float* q : sh->part) (void)hipFree(q);
  for (void* p : {(void*)sh->counts, (void*)sh->send_ids, (void*)sh->recv_ids, (void*)sh->send_emb, (void*)sh->send_w,
                  (void*)sh->hkeys, (void*)sh->hvals, (void*)sh->hslot, (void*)sh->bcnt, (void*)sh->send_ovf,
                  (void*)sh->recv_fix, (void*)sh->srow_emb, (void*)sh->srow_w, (void*)sh->hdr, (void*)sh->recv_ovf,
                  (void*)sh->ovf_emb, (void*)sh->ovf_w})
    if (p) (void)hipFree(p);
  for (int q = 0; q < 2; ++q) {
    for (void* p : {(void*)sh->perm_s[q], (void*)sh->recv_emb_s[q], (void*)sh->recv_w_s[q]})
      if (p) (void)hipFree(p);
    if (sh->ready[q]) (void)hipEventDestroy(sh->ready[q]);
    if (sh->consumed[q]) (void)hipEventDestroy(sh->consumed[q]);
    if (sh->hdr_ev[q]) (void)hipEventDestroy(sh->hdr_ev[q]);
    if (sh->h_hdr_s[q]) (void)hipHostFree(sh->h_hdr_s[q]);
  }
  if (sh->h_counts) (void)hipHostFree(sh->h_counts);
  delete sh;
  return RMX_OK;
}

int shard_fill_synthetic(rmx_shard& sh, uint64_t seed) {
  RMX_HIP(hipSetDevice(sh.ctx->device));
  sh.filled = true;
  hipStream_t s = sh.ctx->stream;
  const float scale = 0.05f * (1.0f / 8388608.0f);
  const int64_t tot = sh.rows_per * sh.rs;
  for (float* q : sh.part) RMX_HIP(hipMemsetAsync(q + tot, 0, sizeof(float) * sh.rs, s));  // the zero row
  for (size_t p = 0; p < sh.part.size(); ++p) {
    const int part = sh.loopback ? (int)p : sh.rank;
    hipLaunchKernelGGL(shard_fill_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, seed, sh.V,
                       sh.rows_per, sh.N, part, sh.k, sh.rs, scale, sh.part[p], owner_perm_of(sh));
    RMX_HIP(hipGetLastError());
  }
  RMX_HIP(hipStreamSynchronize(s));
  return RMX_OK;
}

constexpr int kAutoSkip = 63;

// dedupe = auto: after a deduped batch, skip the step for kAutoSkip batches when it removed < 10 %
void dedupe_auto(rmx_shard& sh, bool dd, int64_t nnz) {
  if (sh.dedupe != 2 || nnz <= 0) return;
  if (dd)
    sh.dedupe_skip = sh.last_sent * 10 > nnz * 9 ? kAutoSkip : 0;
  else if (sh.dedupe_skip > 0)
    --sh.dedupe_skip;
}

// Steps 1-5 of the exchange: fills pull slot `slot` (sh.perm / sh.recv_emb / sh.recv_w) for this
// rank's batch.
// Step 0-1 (dedupe + route) of this rank's batch into pull slot `slot`; *dd = dedupe ran.  cap >= 0: the
// fixed-capacity bucket layout (route_scatter_kernel; cap 0 = every id in the overflow list), cap < 0 the
// dense one; the row slot of an id with no owner is the zero row nfix + nnz (dense: nnz), cleared here.
int shard_route(rmx_shard& sh, hipStream_t s, int64_t nnz, const int32_t* d_ids, int slot, bool* dd_out,
                int64_t cap = -1) {
  const int N = sh.N;
  int st;
  *dd_out = false;
  // test hook (knob "shard_debug_fail_rank" = rank + 1): this rank's route fails as a local error would
  // (out of device memory, ...), so the tests can drive the failed-exchange contract of include/rmx.h
  if (!sh.loopback && tuning_get("shard_debug_fail_rank", 0) == sh.rank + 1) {
    set_error("shard exchange: injected route failure (knob shard_debug_fail_rank)");
    return RMX_E_INVALID;
  }
  const int64_t nfix = cap > 0 ? N * cap : 0;
  if ((st = ensure_batch(sh, nnz, slot, nfix))) return st;
  sh.perm = sh.perm_s[slot];
  sh.recv_emb = sh.recv_emb_s[slot];
  sh.recv_w = sh.recv_w_s[slot];
  const int64_t zslot = nfix + nnz;
  RMX_HIP(hipMemsetAsync(sh.recv_emb + zslot * sh.k, 0, sizeof(float) * sh.k, s));
  RMX_HIP(hipMemsetAsync(sh.recv_w + zslot, 0, sizeof(float), s));
  int32_t* cnt = sh.counts;  // [N] send counts
  RMX_HIP(hipMemsetAsync(sh.counts, 0, sizeof(int32_t) * 4 * N, s));
  // (auto at one rank: off -- no link traffic to save, the duplicates' rows are local reads)
  const bool dd = nnz > 0 && (sh.dedupe == 1 || (sh.dedupe == 2 && sh.N > 1 && sh.dedupe_skip == 0));
  *dd_out = dd;
  int64_t rn = nnz;
  if (nnz <= 0) return RMX_OK;
  // route the batch's ids, or (dedupe) the distinct ids held by the hash set's slots
  const int32_t* rids = d_ids;
  int32_t* rslot = sh.perm;
  if (dd) {
    RMX_HIP(hipMemsetAsync(sh.hkeys, 0xFF, sizeof(int32_t) * sh.cap_hash, s));
    hipLaunchKernelGGL(dedupe_insert_kernel, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, nnz, d_ids,
                       (uint32_t)(sh.cap_hash - 1), 64 - __builtin_ctzll((unsigned long long)sh.cap_hash),
                       sh.hkeys, sh.hslot);
    RMX_HIP(hipGetLastError());
    rids = sh.hkeys;
    rn = sh.cap_hash;
    rslot = sh.hvals;
  }
  const int nb = (int)((rn + kRouteTile - 1) / kRouteTile);
  if ((st = ensure_tiles(sh, nb))) return st;
  const OwnerPerm op = owner_perm_of(sh);
  hipLaunchKernelGGL(route_count_kernel, dim3(nb), dim3(kRouteThreads), 0, s, rn, N, nb, rids, sh.bcnt, op);
  RMX_HIP(hipGetLastError());
  hipLaunchKernelGGL(route_scan_kernel, dim3(N), dim3(1024), 0, s, nb, sh.bcnt, cnt);
  RMX_HIP(hipGetLastError());
  hipLaunchKernelGGL(route_scatter_kernel, dim3(nb), dim3(kRouteThreads), 0, s, rn, N, nb, rids, cnt, sh.bcnt,
                     sh.send_ids, rslot, op, (int32_t)cap, (int32_t)zslot, sh.send_ovf);
  RMX_HIP(hipGetLastError());
  if (dd) {
    hipLaunchKernelGGL(dedupe_perm_kernel, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, nnz, sh.hslot,
                       sh.hvals, sh.perm);
    RMX_HIP(hipGetLastError());
  }
  return RMX_OK;
}

// bucket capacity of the fixed exchange for a routed total nnz: ~1.1 nnz / N (knob "shard_cap_pct", default
// 110) + 64, a multiple of 64 -- uniform ids over N owners stay far inside it (a bucket's spread is
// ~sqrt(nnz / N)); 0 for nnz = 0
int64_t cap_of(const rmx_shard& sh, int64_t nnz) {
  if (nnz <= 0) return 0;
  const int64_t pct = std::max(1, tuning_get("shard_cap_pct", 110));
  const int64_t c = (nnz * pct + 100 * sh.N - 1) / (100 * sh.N) + 64;
  return (c + 63) / 64 * 64;
}

bool fixed_eligible(const rmx_shard& sh) { return sh.N > 1 && !sh.loopback && sh.tr && tuning_get("shard_fixed", 1) != 0; }

// Steps 1-5 with fixed-capacity buckets (N > 1): no host sync.
//   route into [N][cap] (+ overflow list) -> headers + ids to owners (one grouped send / recv, fixed sizes)
//   -> summary to the host (async, read later by shard_resolve) -> owner gather (every peer + own bucket,
//   one launch, bounded by the device counts) -> rows back (fixed sizes).
// The ids of a bucket past cap get their rows in the overflow round, which shard_resolve runs on this
// stream when any rank overflowed (the summary carries the OR of every rank's flag).
int shard_exchange_fixed(rmx_shard& sh, hipStream_t s, int64_t nnz, const int32_t* d_ids, int slot) {
  const int N = sh.N, k = sh.k, me = sh.rank;
  const int64_t cap = sh.cap_next, nfix = N * cap;  // (from the previous exchange: the same on every rank)
  if (nfix >= (int64_t(1) << 31) - nnz - 1) {
    set_error("shard exchange: batch too large for int32 row slots");
    return RMX_E_INVALID;
  }
  bool dd = false;
  int err = shard_route(sh, s, nnz, d_ids, slot, &dd, cap);
  auto keep = [&](int e) {
    if (e && err == RMX_OK) err = e;
    return err == RMX_OK;
  };
  if (err == RMX_OK) keep(ensure_fixed(sh, nfix));
  int32_t* hs = sh.hdr;          // [N][3] sent
  int32_t* hr = sh.hdr + 3 * N;  // [N][3] received
  int32_t* sm = sh.hdr + 6 * N;  // summary [2N + 2]
  if (err == RMX_OK) {
    hipLaunchKernelGGL(fixed_header_kernel, dim3(1), dim3(64), 0, s, N, (int32_t)cap, sh.counts, hs);
    keep(hipGetLastError() == hipSuccess ? RMX_OK : RMX_E_HIP);
  }
  Transport& tr = *sh.tr;
  // (as in the counted exchange: every rank passes every start() / end(), a failed rank posts nothing)
  keep(tr.start());
  for (int o = 0; o < N && err == RMX_OK; ++o) {
    if (o == me) continue;
    if (keep(tr.send(hs + 3 * o, 3 * sizeof(int32_t), o, s)) && (cap == 0 || keep(tr.send(sh.send_ids + o * cap, sizeof(int32_t) * cap, o, s))) &&
        keep(tr.recv(hr + 3 * o, 3 * sizeof(int32_t), o, s)) && cap > 0)
      keep(tr.recv(sh.recv_fix + o * cap, sizeof(int32_t) * cap, o, s));
  }
  keep(tr.end(s));
  if (err == RMX_OK) {
    hipLaunchKernelGGL(fixed_summary_kernel, dim3(1), dim3(64), 0, s, N, me, sh.counts, hs, hr, sm);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(sh.h_hdr_s[slot], sm, sizeof(int32_t) * (2 * N + 2), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipEventRecord(sh.hdr_ev[slot], s) != hipSuccess) {
      set_error("shard exchange: the summary's device-to-host copy failed");
      keep(RMX_E_HIP);
    }
  }
  if (err == RMX_OK && nfix > 0) {
    const int64_t threads = (k == 16 && sh.rs == 32) ? nfix * 8 : nfix;
    hipLaunchKernelGGL(fixed_gather_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, N, me,
                       (int32_t)cap, k, sh.rs, sh.counts, hr, sh.send_ids, sh.recv_fix, sh.part[0], sh.srow_emb,
                       sh.srow_w, sh.recv_emb, sh.recv_w);
    keep(hipGetLastError() == hipSuccess ? RMX_OK : RMX_E_HIP);
  }
  keep(tr.start());
  for (int o = 0; o < N && err == RMX_OK && cap > 0; ++o) {
    if (o == me) continue;
    if (keep(tr.send(sh.srow_emb + o * cap * k, sizeof(float) * cap * k, o, s)) &&
        keep(tr.send(sh.srow_w + o * cap, sizeof(float) * cap, o, s)) &&
        keep(tr.recv(sh.recv_emb + o * cap * k, sizeof(float) * cap * k, o, s)))
      keep(tr.recv(sh.recv_w + o * cap, sizeof(float) * cap, o, s));
  }
  keep(tr.end(s));
  sh.unresolved[slot] = err == RMX_OK;
  sh.last_fixed = err == RMX_OK ? slot : -1;
  sh.last_sent_dev = false;
  sh.slot_stream[slot] = s;
  sh.slot_cap[slot] = cap;
  sh.slot_n[slot] = nnz;
  sh.slot_dd[slot] = dd;
  return err;
}

// The overflow check of a fixed exchange in slot `slot` (a no-op once done): waits for its summary --
// normally long on the host already -- and, when any rank overflowed, runs the counted overflow round on
// the exchange's stream: overflow ids to owners, owner gather, rows back into [N * cap, ...).  Every rank
// calls this for the same exchanges in the same order (the next exchange and the slot's forward both
// resolve first), so the rounds pair up.  *ran = the overflow round ran (the slot's rows changed).
int shard_resolve(rmx_shard& sh, int slot, bool* ran = nullptr) {
  if (ran) *ran = false;
  if (!sh.unresolved[slot]) return RMX_OK;
  sh.unresolved[slot] = false;
  RMX_HIP(hipEventSynchronize(sh.hdr_ev[slot]));
  const int N = sh.N, k = sh.k, me = sh.rank;
  const int32_t* h = sh.h_hdr_s[slot];
  const int64_t cap = sh.slot_cap[slot], nfix = N * cap;
  {  // (dedupe auto needs this exchange's sent total)
    const int64_t keep_sent = sh.last_sent;
    sh.last_sent = 0;
    for (int o = 0; o < N; ++o) sh.last_sent += h[o];
    dedupe_auto(sh, sh.slot_dd[slot], sh.slot_n[slot]);
    if (sh.last_fixed != slot) sh.last_sent = keep_sent;
  }
  sh.cap_next = cap_of(sh, h[2 * N + 1]);  // the next exchange's capacity (identical on every rank)
  if (!h[2 * N]) return RMX_OK;
  ++sh.rounds2;
  if (ran) *ran = true;
  hipStream_t s = sh.slot_stream[slot];
  std::vector<int64_t> ho(N), hro(N), os(N + 1, 0), ros(N + 1, 0);
  for (int o = 0; o < N; ++o) {
    ho[o] = std::max<int64_t>(0, h[o] - cap);
    hro[o] = o == me ? 0 : std::max<int64_t>(0, h[N + o] - cap);
    os[o + 1] = os[o] + ho[o];     // the scatter's overflow order: buckets in owner order
    ros[o + 1] = ros[o] + hro[o];  // the peers' overflow requests, in peer order
  }
  int err = ensure_ovf(sh, ros[N]);
  auto keep = [&](int e) {
    if (e && err == RMX_OK) err = e;
    return err == RMX_OK;
  };
  float* remb = sh.recv_emb_s[slot];
  float* rw = sh.recv_w_s[slot];
  Transport& tr = *sh.tr;
  keep(tr.start());
  for (int o = 0; o < N && err == RMX_OK; ++o) {
    if (o == me) continue;
    if (ho[o]) keep(tr.send(sh.send_ovf + os[o], sizeof(int32_t) * ho[o], o, s));
    if (hro[o] && err == RMX_OK) keep(tr.recv(sh.recv_ovf + ros[o], sizeof(int32_t) * hro[o], o, s));
  }
  keep(tr.end(s));
  if (err == RMX_OK) keep(launch_owner_gather(s, ros[N], k, sh.rs, sh.recv_ovf, sh.part[0], sh.ovf_emb, sh.ovf_w));
  if (err == RMX_OK)
    keep(launch_owner_gather(s, ho[me], k, sh.rs, sh.send_ovf + os[me], sh.part[0], remb + (nfix + os[me]) * k,
                             rw + nfix + os[me]));
  keep(tr.start());
  for (int o = 0; o < N && err == RMX_OK; ++o) {
    if (o == me) continue;
    if (hro[o] && keep(tr.send(sh.ovf_emb + ros[o] * k, sizeof(float) * hro[o] * k, o, s)))
      keep(tr.send(sh.ovf_w + ros[o], sizeof(float) * hro[o], o, s));
    if (ho[o] && err == RMX_OK && keep(tr.recv(remb + (nfix + os[o]) * k, sizeof(float) * ho[o] * k, o, s)))
      keep(tr.recv(rw + nfix + os[o], sizeof(float) * ho[o], o, s));
  }
  keep(tr.end(s));
  if (err == RMX_OK && sh.ready[slot]) keep(hipEventRecord(sh.ready[slot], s) == hipSuccess ? RMX_OK : RMX_E_HIP);
  // the scratch this round read (send_ovf, recv_ovf, ovf_*) is free once s passes here: the next exchange,
  // on whatever stream, waits for it (shard_exchange)
  if (!sh.ovf_done && hipEventCreateWithFlags(&sh.ovf_done, hipEventDisableTiming) != hipSuccess) sh.ovf_done = nullptr;
  if (sh.ovf_done && hipEventRecord(sh.ovf_done, s) == hipSuccess)
    sh.ovf_pending = true;
  else
    keep(RMX_E_HIP);
  if (err != RMX_OK) sh.failed = true;
  return err;
}

// every pending overflow check, oldest pull first (before an exchange reuses the scratch buffers)
int shard_resolve_all(rmx_shard& sh) {
  int st = RMX_OK;
  for (int q = 0; q < 2; ++q)
    if (sh.unresolved[q] && !st) st = shard_resolve(sh, q);
  return st;
}

// Steps 1-5 of the exchange: fills pull slot `slot` (sh.perm / sh.recv_emb / sh.recv_w) for this
// rank's batch.
int shard_exchange(rmx_shard& sh, hipStream_t s, int64_t nnz, const int32_t* d_ids, int slot = 0) {
  const int N = sh.N, k = sh.k;
  int st;
  bool dd = false;
  if (sh.failed) {
    set_error("shard exchange: an earlier exchange failed on this rank, so its collectives no longer pair up "
              "with its peers'; abort the shard (rmx_shard_abort) and create a new one");
    return RMX_E_COMM;
  }
  if ((st = shard_resolve_all(sh))) return st;  // a pending overflow round uses the scratch below
  if (sh.ovf_pending) {  // ... possibly on another stream
    RMX_HIP(hipStreamWaitEvent(s, sh.ovf_done, 0));
    sh.ovf_pending = false;
  }
  if (fixed_eligible(sh)) {
    if (sh.comm_state.load() != 0) {
      set_error("shard exchange: the communicator was aborted (rmx_shard_abort)");
      return RMX_E_COMM;
    }
    st = shard_exchange_fixed(sh, s, nnz, d_ids, slot);
    if (st) sh.failed = true;
    return st;
  }
  sh.last_fixed = -1;
  if (N == 1 && !sh.loopback && sh.dedupe != 1) {
    // one rank, no dedupe (auto is off at one rank): identity routing, one gather pass, no host sync
    if ((st = ensure_batch(sh, nnz, slot))) return st;
    sh.perm = sh.perm_s[slot];
    sh.recv_emb = sh.recv_emb_s[slot];
    sh.recv_w = sh.recv_w_s[slot];
    sh.last_sent = nnz;
    sh.last_sent_dev = false;
    if (nnz <= 0) return RMX_OK;
    const int64_t threads = (k == 16 && sh.rs == 32) ? nnz * 8 : nnz;
    hipLaunchKernelGGL(own_gather_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, nnz, k, sh.rs,
                       d_ids, sh.part[0], sh.recv_emb, sh.recv_w, sh.perm, owner_perm_of(sh));
    RMX_HIP(hipGetLastError());
    return RMX_OK;
  }
  const int route_err = shard_route(sh, s, nnz, d_ids, slot, &dd);
  int32_t* cnt = sh.counts;       // [N] send counts
  int32_t* rcnt = sh.counts + N;  // [N] recv counts
  if (sh.loopback) {
    if (route_err) return route_err;
    // loopback: partition o serves bucket o in place
    RMX_HIP(hipMemcpyAsync(sh.h_counts, cnt, sizeof(int32_t) * N, hipMemcpyDeviceToHost, s));
    RMX_HIP(hipStreamSynchronize(s));
    int64_t off = 0;
    sh.last_sent = 0;
    sh.last_sent_dev = false;
    for (int o = 0; o < N; ++o) sh.last_sent += sh.h_counts[o];
    dedupe_auto(sh, dd, nnz);
    for (int o = 0; o < N; ++o) {
      const int64_t c = sh.h_counts[o];
      if ((st = launch_owner_gather(s, c, k, sh.rs, sh.send_ids + off, sh.part[o], sh.recv_emb + off * k,
                                    sh.recv_w + off)))
        return st;
      off += c;
    }
    return RMX_OK;
  }
  if (N == 1) {
    if (route_err) return route_err;
    // one rank: no exchange.  The bucket is this rank's own; its size (nnz, or the distinct ids
    // when deduplicating) stays on the device and bounds the gather there -- no host sync.
    sh.last_sent = nnz;
    sh.last_sent_dev = dd;
    dedupe_auto(sh, dd, nnz);
    // (the device count also bounds a batch holding ids outside [0, V), which route no row)
    return launch_owner_gather(s, nnz, k, sh.rs, sh.send_ids, sh.part[0], sh.recv_emb, sh.recv_w, cnt);
  }
  if (sh.comm_state.load() != 0) {
    set_error("shard exchange: the communicator was aborted (rmx_shard_abort)");
    return RMX_E_COMM;
  }
  Transport& tr = *sh.tr;
  const int me = sh.rank;
  // From here every rank passes all three start() / end() rendezvous, also after a local error
  // (the route above, a transport call, the owner-side buffers): a failed rank posts no more ops,
  // so its peers fail the receives they expected from it with RMX_E_COMM at once, instead of
  // waiting out the group timeout that would break the group for good.  (RCCL has no such
  // recovery: a peer's unmatched receive there waits for the communicator's abort.)
  int err = route_err;
  auto keep = [&](int e) {
    if (e && err == RMX_OK) err = e;
    return err == RMX_OK;
  };
  // 2. counts: one int to every peer, then one D2H of the 2N counts (the only host sync: the
  //    transport needs host-side message sizes); this rank's own entry is a local copy
  keep(tr.start());
  for (int o = 0; o < N && err == RMX_OK; ++o) {
    if (o == me) continue;
    if (keep(tr.send(cnt + o, sizeof(int32_t), o, s))) keep(tr.recv(rcnt + o, sizeof(int32_t), o, s));
  }
  keep(tr.end(s));
  int32_t* hc = sh.h_counts;
  int32_t* hr = sh.h_counts + N;
  if (err == RMX_OK) {
    if (hipMemcpyAsync(sh.h_counts, cnt, sizeof(int32_t) * 2 * N, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      set_error("shard exchange: the counts' device-to-host copy failed");
      keep(RMX_E_HIP);
    }
  }
  // an abort while this thread waited for the counts: post nothing more (the comm is torn down)
  if (err == RMX_OK && sh.comm_state.load() != 0) {
    set_error("shard exchange: the communicator was aborted (rmx_shard_abort)");
    keep(RMX_E_COMM);
  }
  if (err != RMX_OK) std::fill(sh.h_counts, sh.h_counts + 2 * N, 0);  // post nothing from here
  hr[me] = hc[me];
  sh.last_sent = 0;
  sh.last_sent_dev = false;
  for (int o = 0; o < N; ++o) sh.last_sent += hc[o];
  dedupe_auto(sh, dd, nnz);
  // Owner-side buffers hold the PEERS' requests only: peer o's range starts at ro(o) = sum of
  // hr[p] over p < o, p != me.  The own bucket never goes through the transport: its rows are
  // gathered straight into their requester-order slots [so_me, so_me + hc[me]).
  int64_t npeer = 0, so_me = 0;
  for (int o = 0; o < N; ++o) {
    if (o != me) npeer += hr[o];
    if (o < me) so_me += hc[o];
  }
  if (err == RMX_OK) keep(ensure_recv(sh, npeer));
  // 3. ids to owners
  keep(tr.start());
  for (int64_t o = 0, so = 0, ro = 0; o < N && err == RMX_OK; so += hc[o], ro += (o == me ? 0 : hr[o]), ++o) {
    if (o == me) continue;
    if (hc[o]) keep(tr.send(sh.send_ids + so, sizeof(int32_t) * hc[o], (int)o, s));
    if (hr[o] && err == RMX_OK) keep(tr.recv(sh.recv_ids + ro, sizeof(int32_t) * hr[o], (int)o, s));
  }
  keep(tr.end(s));
  // 4. owner gather: every peer's request in one launch, then the own bucket
  if (err == RMX_OK) keep(launch_owner_gather(s, npeer, k, sh.rs, sh.recv_ids, sh.part[0], sh.send_emb, sh.send_w));
  if (err == RMX_OK)
    keep(launch_owner_gather(s, hc[me], k, sh.rs, sh.send_ids + so_me, sh.part[0], sh.recv_emb + so_me * k,
                             sh.recv_w + so_me));
  // 5. rows back, into the requester's bucket order
  keep(tr.start());
  for (int64_t o = 0, so = 0, ro = 0; o < N && err == RMX_OK; so += hc[o], ro += (o == me ? 0 : hr[o]), ++o) {
    if (o == me) continue;
    if (hr[o] && keep(tr.send(sh.send_emb + ro * k, sizeof(float) * hr[o] * k, (int)o, s)))
      keep(tr.send(sh.send_w + ro, sizeof(float) * hr[o], (int)o, s));
    if (hc[o] && err == RMX_OK && keep(tr.recv(sh.recv_emb + so * k, sizeof(float) * hc[o] * k, (int)o, s)))
      keep(tr.recv(sh.recv_w + so, sizeof(float) * hc[o], (int)o, s));
  }
  keep(tr.end(s));
  //  as on the fixed path: a failed exchange leaves this rank out of step with its peers, so
  // every later exchange on the shard fails at once (include/rmx.h)
  if (err != RMX_OK) sh.failed = true;
  return err;
}

// The in-place read at one rank (no dedupe, k = 16 line rows): fills perm_s[slot] with the batch's
// partition rows.  Returns false (nothing done) when the shard does not qualify.
bool direct_eligible(const rmx_shard& sh) {
  return sh.N == 1 && !sh.loopback && sh.dedupe != 1 && sh.k == 16 && sh.rs == 32 && sh.rows_per < (int64_t(1) << 31);
}

int shard_map_rows(rmx_shard& sh, hipStream_t s, int64_t nnz, const int32_t* d_ids, int slot) {
  int st;
  sh.last_fixed = -1;
  if ((st = ensure_batch(sh, nnz, slot))) return st;
  sh.last_sent = nnz;
  sh.last_sent_dev = false;
  if (nnz <= 0) return RMX_OK;
  hipLaunchKernelGGL(own_rows_kernel, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, nnz, d_ids,
                     (int32_t)sh.rows_per, sh.perm_s[slot], owner_perm_of(sh));
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// the forward of a directly-mapped slot: in place for models that read line rows, else the rows
// are copied out first (owner gather through the mapped rows) and the forward runs on them in batch
// order (implicit ids n)
int forward_direct(rmx_model& m, rmx_shard& sh, hipStream_t s, int B, const int32_t* rows, int slot, float* d_out) {
  FwdInputs in;
  in.B = B;
  in.dtype = kF32;
  in.beta = m.beta;
  in.out = d_out;
  if (model_reads_lines(m)) {
    in.ids = rows;
    in.table = sh.part[0];
    in.wtab = sh.part[0] + sh.k;
    in.ld = sh.rs;
    in.wld = sh.rs;
    return model_forward(m, s, in);
  }
  const int64_t n = (int64_t)B * m.F;
  int st;
  {
    StageTimer t(m, s, "shard_exchange");
    if ((st = launch_owner_gather(s, n, sh.k, sh.rs, rows, sh.part[0], sh.recv_emb_s[slot], sh.recv_w_s[slot])))
      return st;
    // the rows are in batch order now: the slot's row list becomes the identity (stream-ordered after
    // the gather read it), so the forward runs the same id-array kernels as every other path
    if (n > 0) {
      hipLaunchKernelGGL(iota_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n,
                         const_cast<int32_t*>(rows));
      RMX_HIP(hipGetLastError());
    }
  }
  in.ids = rows;
  in.table = sh.recv_emb_s[slot];
  in.wtab = sh.recv_w_s[slot];
  return model_forward(m, s, in);
}

}  // namespace rmx

// ------------------------------------------------------------------ C ABI --
using namespace rmx;

extern "C" int rmx_comm_unique_id(void* out, size_t cap) {
  if (!out || cap < sizeof(ncclUniqueId)) {
    set_error("rmx_comm_unique_id: buffer must hold RMX_UNIQUE_ID_BYTES bytes");
    return RMX_E_INVALID;
  }
  ncclUniqueId id;
  RMX_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
  return RMX_OK;
}

extern "C" int rmx_shard_create(rmx_ctx* ctx, int64_t num_rows, int embedding_dim, int nranks, int rank,
                                const void* unique_id, rmx_shard** out) {
  if (!ctx || !out) {
    set_error("rmx_shard_create: bad args");
    return RMX_E_INVALID;
  }
  return shard_create(ctx, num_rows, embedding_dim, nranks, rank, unique_id, nullptr, out);
}

extern "C" int rmx_group_create(int nranks, rmx_group** out) {
  if (!out || nranks < 1 || nranks > kMaxRanks) {
    set_error("rmx_group_create: need 1 <= nranks <= 64");
    return RMX_E_INVALID;
  }
  auto* g = new rmx_group();
  g->N = nranks;
  g->posted.resize((size_t)nranks * nranks);
  g->ev_send.assign(nranks, nullptr);
  g->ev_done.assign(nranks, nullptr);
  g->attached.assign(nranks, 0);
  *out = g;
  return RMX_OK;
}

extern "C" int rmx_group_destroy(rmx_group* g) {
  if (g) group_unref(g);  // the group lives on until its last shard is destroyed
  return RMX_OK;
}

extern "C" int rmx_shard_create_group(rmx_ctx* ctx, int64_t num_rows, int embedding_dim, rmx_group* group, int rank,
                                      rmx_shard** out) {
  if (!ctx || !out || !group) {
    set_error("rmx_shard_create_group: bad args");
    return RMX_E_INVALID;
  }
  return shard_create(ctx, num_rows, embedding_dim, group->N, rank, nullptr, group, out);
}

extern "C" int rmx_shard_destroy(rmx_shard* sh) { return shard_destroy(sh); }

extern "C" int rmx_shard_abort(rmx_shard* sh) {
  if (!sh) {
    rmx::set_error("rmx_shard_abort: null shard");
    return RMX_E_INVALID;
  }
  int live = 0;  // claim the communicator (a destroy or an earlier abort got it first: nothing to do)
  if (!sh->comm || !sh->comm_state.compare_exchange_strong(live, 1)) return RMX_OK;
  // no exchange bracket in flight on the host (RcclTransport): its calls finish, later brackets see the
  // state and post nothing.  A thread blocked inside an RCCL call keeps the lock: after the bounded wait
  // the abort goes ahead anyway, which is the case ncclCommAbort exists for.
  const bool locked = sh->tr_mu.try_lock_for(std::chrono::seconds(5));
  const ncclResult_t r = ncclCommAbort(sh->comm);
  if (locked) sh->tr_mu.unlock();
  if (r != ncclSuccess) {
    rmx::set_error(std::string("rmx_shard_abort: ") + ncclGetErrorString(r));
    return RMX_E_COMM;
  }
  return RMX_OK;
}

extern "C" int rmx_shard_fill_synthetic(rmx_shard* sh, uint64_t seed) {
  if (!sh) {
    set_error("rmx_shard_fill_synthetic: NULL shard");
    return RMX_E_INVALID;
  }
  return shard_fill_synthetic(*sh, seed);
}

extern "C" int64_t rmx_shard_local_rows(const rmx_shard* sh) { return sh ? sh->rows_per : -1; }

extern "C" int rmx_shard_set_owner_hash(rmx_shard* sh, uint64_t key) {
  if (!sh) {
    set_error("rmx_shard_set_owner_hash: NULL shard");
    return RMX_E_INVALID;
  }
  std::lock_guard<std::mutex> lk(sh->mu);
  if (sh->filled) {
    set_error("rmx_shard_set_owner_hash: set the owner function before the rows are filled");
    return RMX_E_INVALID;
  }
  sh->owner_key = key;
  return RMX_OK;
}

extern "C" int64_t rmx_shard_owner_of(const rmx_shard* sh, int64_t id) {
  if (!sh || id < 0 || id >= sh->V) return -1;
  return owner_perm(id, owner_perm_of(*sh), false) % sh->N;
}

extern "C" int64_t rmx_owner_hash(uint64_t key, int64_t num_rows, int nranks, int64_t id, int64_t* local_row) {
  if (num_rows < 1 || num_rows >= (int64_t(1) << 31) || nranks < 1 || id < 0 || id >= num_rows) return -1;
  const int64_t p = owner_perm(id, owner_perm_of(key, num_rows), false);
  if (local_row) *local_row = p / nranks;
  return p % nranks;
}

extern "C" int64_t rmx_shard_overflow_rounds(const rmx_shard* sh) { return sh ? sh->rounds2 : -1; }

extern "C" int rmx_shard_set_batch_hint(rmx_shard* sh, int64_t nnz) {
  if (!sh || nnz < 0) {
    set_error("rmx_shard_set_batch_hint: NULL shard or negative nnz");
    return RMX_E_INVALID;
  }
  std::lock_guard<std::mutex> lk(sh->mu);
  // the first fixed exchange's bucket capacity (later ones take it from the previous exchange's summary);
  // every rank passes the same value, so the message sizes pair up
  sh->cap_next = cap_of(*sh, nnz);
  return RMX_OK;
}

extern "C" int rmx_shard_set_dedupe(rmx_shard* sh, int on) {
  if (!sh) {
    set_error("rmx_shard_set_dedupe: NULL shard");
    return RMX_E_INVALID;
  }
  if (on < 0 || on > 2) {
    set_error("rmx_shard_set_dedupe: on must be 0 (off), 1 (on) or 2 (auto)");
    return RMX_E_INVALID;
  }
  std::lock_guard<std::mutex> lk(sh->mu);
  sh->dedupe = on;
  sh->dedupe_skip = 0;
  return RMX_OK;
}

extern "C" int64_t rmx_shard_last_sent(const rmx_shard* sh) {
  if (!sh) return -1;
  if (sh->last_fixed >= 0) {  // the last exchange was a fixed one: its summary (a local wait, no collective)
    const int q = sh->last_fixed;
    if (hipSetDevice(sh->ctx->device) != hipSuccess || hipEventSynchronize(sh->hdr_ev[q]) != hipSuccess) return -1;
    int64_t t = 0;
    for (int o = 0; o < sh->N; ++o) t += sh->h_hdr_s[q][o];
    sh->last_sent = t;
    sh->last_fixed = -1;
    return t;
  }
  if (sh->last_sent_dev) {  // one rank, deduplicated: the distinct count is counts[0] on the device
    int32_t c = 0;
    if (hipSetDevice(sh->ctx->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(&c, sh->counts, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess)
      return -1;
    sh->last_sent = c;
    sh->last_sent_dev = false;
  }
  return sh->last_sent;
}

extern "C" int rmx_shard_gather(rmx_shard* sh, int64_t n, const int32_t* d_ids, float* d_w, float* d_emb,
                                void* stream) {
  if (!sh || (!d_ids && n > 0) || n < 0 || (n > 0 && (!d_w || !d_emb))) {
    set_error("rmx_shard_gather: bad args");
    return RMX_E_INVALID;
  }
  RMX_HIP(hipSetDevice(sh->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : sh->ctx->stream;
  ShardUse use(*sh, s);
  if (use.st) return use.st;
  if (sh->slot_nnz[0] >= 0) {
    set_error("rmx_shard_gather: pull slot 0 holds a pull no rmx_forward_pulled has consumed yet");
    return RMX_E_INVALID;
  }
  if (sh->consumed_rec[0]) RMX_HIP(hipStreamWaitEvent(s, sh->consumed[0], 0));
  int st = shard_exchange(*sh, s, n, d_ids, 0);
  if (st) return st;
  // un-permute into id order: d_emb[i] = recv_emb[perm[i]]; then the overflow check (a fixed exchange):
  // when the overflow round ran, the un-permute runs again over the completed rows
  for (int pass = 0; pass < 2; ++pass) {
    if (n > 0) {
      const int64_t threads = sh->k == 16 ? n * 4 : n;
      hipLaunchKernelGGL(unpermute_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, n, sh->k,
                         sh->perm, sh->recv_emb, sh->recv_w, d_emb, d_w);
      RMX_HIP(hipGetLastError());
    }
    bool ran = false;
    if (pass == 0 && ((st = shard_resolve(*sh, 0, &ran)) || !ran)) return st;
  }
  return RMX_OK;
}

// Pull (exchange) a batch into slot `slot` on `stream`, then let rmx_forward_pulled consume it on
// another stream: batch i + 1's exchange runs beside batch i's forward (ParRecModel's pull* and the
// model forward are separate calls in the reference too: ParRecModel.scala:165-199 then :279-306).
extern "C" int rmx_shard_pull(rmx_shard* sh, int64_t n, const int32_t* d_ids, int slot, void* stream) {
  if (!sh || n < 0 || (!d_ids && n > 0) || slot < 0 || slot > 1) {
    set_error("rmx_shard_pull: bad args (slot must be 0 or 1)");
    return RMX_E_INVALID;
  }
  RMX_HIP(hipSetDevice(sh->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : sh->ctx->stream;
  ShardUse use(*sh, s);  // the exchange's internal buffers: one pull at a time
  if (use.st) return use.st;
  if (sh->slot_nnz[slot] >= 0) {
    set_error("rmx_shard_pull: slot " + std::to_string(slot) + " holds a pull no forward has consumed yet");
    return RMX_E_INVALID;
  }
  for (int q = 0; q < 2; ++q)
    if (!sh->ready[q]) {
      RMX_HIP(hipEventCreateWithFlags(&sh->ready[q], hipEventDisableTiming));
      RMX_HIP(hipEventCreateWithFlags(&sh->consumed[q], hipEventDisableTiming));
    }
  // the slot's previous forward must have read it before the exchange overwrites it
  if (sh->consumed_rec[slot]) RMX_HIP(hipStreamWaitEvent(s, sh->consumed[slot], 0));
  const bool direct = direct_eligible(*sh);
  int st = direct ? shard_map_rows(*sh, s, n, d_ids, slot) : shard_exchange(*sh, s, n, d_ids, slot);
  if (st) return st;
  sh->slot_direct[slot] = direct;
  RMX_HIP(hipEventRecord(sh->ready[slot], s));
  sh->slot_nnz[slot] = n;
  return RMX_OK;
}

extern "C" int rmx_forward_pulled(rmx_model* m, rmx_shard* sh, int32_t B, int slot, float* d_out, void* stream) {
  if (!m || !sh || !d_out || B < 0 || slot < 0 || slot > 1 || !m->ctx) {
    set_error("rmx_forward_pulled: bad args (slot must be 0 or 1)");
    return RMX_E_INVALID;
  }
  if (!m->params_ready && m->mats_len > 0) {
    set_error("rmx_forward_pulled: call rmx_model_set_mats first");
    return RMX_E_INVALID;
  }
  if (!m->beta_set) {
    set_error("rmx_forward_pulled: call rmx_model_set_bias first");
    return RMX_E_INVALID;
  }
  if (m->precision != RMX_DTYPE_F32) {
    set_error("rmx_forward_pulled: sharded tables are fp32 (model precision must be RMX_DTYPE_F32)");
    return RMX_E_INVALID;
  }
  if (m->type != RMX_MODEL_LR && sh->k != m->k) {
    set_error("rmx_forward_pulled: table embedding_dim differs from the model's");
    return RMX_E_SHAPE;
  }
  RMX_HIP(hipSetDevice(m->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : m->ctx->stream;
  int32_t* perm;
  float *emb, *w;
  {
    std::lock_guard<std::mutex> lk(sh->mu);
    if (sh->slot_nnz[slot] != (int64_t)B * m->F) {
      set_error(sh->slot_nnz[slot] < 0 ? "rmx_forward_pulled: nothing pulled into slot " + std::to_string(slot)
                                       : "rmx_forward_pulled: the slot holds " + std::to_string(sh->slot_nnz[slot]) +
                                             " ids, not batch * nFields");
      return sh->slot_nnz[slot] < 0 ? RMX_E_INVALID : RMX_E_SHAPE;
    }
    // the slot's overflow check (normally its summary is long on the host; the overflow round, when
    // any rank needs it, runs on the pull's stream and re-records ready)
    const int rst = shard_resolve(*sh, slot);
    if (rst) return rst;
    RMX_HIP(hipStreamWaitEvent(s, sh->ready[slot], 0));
    perm = sh->perm_s[slot];
    emb = sh->recv_emb_s[slot];
    w = sh->recv_w_s[slot];
  }
  int st;
  if (sh->slot_direct[slot]) {
    ModelUse use(*m, s);
    if (use.st) return use.st;
    st = forward_direct(*m, *sh, s, B, perm, slot, d_out);
  } else {
    ModelUse use(*m, s);
    if (use.st) return use.st;
    FwdInputs in;
    in.B = B;
    in.ids = perm;
    in.table = emb;
    in.wtab = w;
    in.dtype = kF32;
    in.beta = m->beta;
    in.out = d_out;
    st = model_forward(*m, s, in);
  }
  std::lock_guard<std::mutex> lk(sh->mu);
  RMX_HIP(hipEventRecord(sh->consumed[slot], s));
  sh->consumed_rec[slot] = true;
  sh->slot_nnz[slot] = -1;
  return st;
}

extern "C" int rmx_forward_ids_sharded(rmx_model* m, rmx_shard* sh, int32_t B, const int32_t* d_ids, float* d_out,
                                       void* stream) {
  if (!m || !sh || !d_out || B < 0 || (!d_ids && B > 0) || !m->ctx) {
    set_error("rmx_forward_ids_sharded: bad args");
    return RMX_E_INVALID;
  }
  if (!m->params_ready && m->mats_len > 0) {
    set_error("rmx_forward_ids_sharded: call rmx_model_set_mats first");
    return RMX_E_INVALID;
  }
  if (!m->beta_set) {
    set_error("rmx_forward_ids_sharded: call rmx_model_set_bias first");
    return RMX_E_INVALID;
  }
  if (m->precision != RMX_DTYPE_F32) {
    set_error("rmx_forward_ids_sharded: sharded tables are fp32 (model precision must be RMX_DTYPE_F32)");
    return RMX_E_INVALID;
  }
  if (m->type != RMX_MODEL_LR && sh->k != m->k) {
    set_error("rmx_forward_ids_sharded: table embedding_dim differs from the model's");
    return RMX_E_SHAPE;
  }
  RMX_HIP(hipSetDevice(m->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : m->ctx->stream;
  ShardUse suse(*sh, s);  // lock order: shard, then model
  if (suse.st) return suse.st;
  ModelUse use(*m, s);
  if (use.st) return use.st;
  if (sh->slot_nnz[0] >= 0) {
    set_error("rmx_forward_ids_sharded: pull slot 0 holds a pull no rmx_forward_pulled has consumed yet");
    return RMX_E_INVALID;
  }
  if (sh->consumed_rec[0]) RMX_HIP(hipStreamWaitEvent(s, sh->consumed[0], 0));
  int st;
  if (direct_eligible(*sh)) {
    // one rank: the batch's partition rows, then the forward reads the lines in place
    {
      StageTimer t(*m, s, "shard_exchange");
      st = shard_map_rows(*sh, s, (int64_t)B * m->F, d_ids, 0);
    }
    if (st) return st;
    return forward_direct(*m, *sh, s, B, sh->perm_s[0], 0, d_out);
  }
  {
    StageTimer t(*m, s, "shard_exchange");
    st = shard_exchange(*sh, s, (int64_t)B * m->F, d_ids, 0);
  }
  if (st) return st;
  if (m->timing) ++m->timed_calls;  // model_forward counts it again; undone below
  FwdInputs in;
  in.B = B;
  in.ids = sh->perm;
  in.table = sh->recv_emb;
  in.wtab = sh->recv_w;
  in.dtype = kF32;
  in.beta = m->beta;
  in.out = d_out;
  st = model_forward(*m, s, in);
  if (m->timing) --m->timed_calls;
  if (st) return st;
  // a fixed exchange's overflow check comes after the forward is queued (the host waits on a summary the
  // GPU produced before the rows even moved); when the overflow round runs, the forward runs again.  The
  // round is part of the exchange's stage (it used to fall outside every timer); the re-run
  // forward's kernels add to their own stages, over the same call count.
  bool ran = false;
  {
    StageTimer t(*m, s, "shard_exchange");
    st = shard_resolve(*sh, 0, &ran);
  }
  if (st || !ran) return st;
  if (m->timing) ++m->timed_calls;
  st = model_forward(*m, s, in);
  if (m->timing) --m->timed_calls;
  return st;
}
