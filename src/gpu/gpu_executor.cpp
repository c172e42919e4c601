#include "gpu/gpu_executor.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <thread>

#include "core/timing.hpp"
#include "fft/fft_plan.hpp"
#include "gpu/device_comm.hpp"
#include "spfft/exceptions.hpp"

namespace spfft {



namespace {
int env_int(const char* name, int dflt, int lo, int hi) {
  const char* e = std::getenv(name);
  if (!e || !*e) return dflt;
  const int v = std::atoi(e);
  return v < lo ? lo : (v > hi ? hi : v);
}
}  // namespace

template <typename T>
template <typename U>
U* GpuExecutor<T>::upload(std::unique_ptr<DeviceBuffer>& buf, const std::vector<U>& v) {
  if (v.empty()) return nullptr;
  buf.reset(new DeviceBuffer(v.size() * sizeof(U)));
  gpu_check(hipMemcpy(buf->data(), v.data(), v.size() * sizeof(U), hipMemcpyHostToDevice),
            "hipMemcpy");
  return buf->data<U>();
}

template <typename T>
GpuExecutor<T>::GpuExecutor(std::shared_ptr<GridImpl<T>> grid,
                            std::shared_ptr<const IndexPlan> plan)
    : grid_(std::move(grid)), plan_(std::move(plan)), deviceId_(grid_->device_id()) {
  DeviceGuard guard(deviceId_);
  const IndexPlan& p = *plan_;
  const bool distributed = p.size > 1;
  floatExchange_ = distributed && is_exchange_float(grid_->exchange_type());
  const int stickElemBytes = floatExchange_ ? sizeof(cx<float>) : sizeof(cx<T>);
  layout_ = make_exchange_layout(p, distributed && is_exchange_buffered(grid_->exchange_type()),
                                 aligned_row_pad(p.dimZ, stickElemBytes));
  interStride_ = p.dimY + aligned_row_pad(p.dimY, sizeof(cx<T>));
  poison_ = env_int("SPFFT_POISON", 0, 0, 1) != 0;
  // opt-in: on ROCm 7.2 a replayed graph was measured slower than direct
  // launches in stream-ordered use (profiles/README.md, session 6)
  graphsEnabled_ = env_int("SPFFT_GRAPH", 0, 0, 1) != 0;
  if (layout_.stickTotal > grid_->slot_elements(GridImpl<T>::kStickSide) ||
      layout_.slabTotal > grid_->slot_elements(GridImpl<T>::kSlabSide))
    throw InvalidParameterError();
  {
    // plane ranges of the y/x stages that fit the grid's (capped) intermediate
    const long long perPlane = static_cast<long long>(p.num_columns()) * interStride_;
    if (perPlane >= (1LL << 31)) throw InvalidParameterError();  // 32-bit row offsets
    const int L = std::max(p.local_planes(), 1);
    const long long cap = grid_->device_slot_elements(GridImpl<T>::kInter);
    interPlanes_ = perPlane > 0 ? static_cast<int>(std::min<long long>(L, std::max(1LL, cap / perPlane))) : L;
  }
  setup_long_axes();
  // Backward z -> y hand-off through the Infinity Cache: a single rank's z
  // stage writes the stick array that its y stage reads next. With the default
  // cache policy on both sides (instead of streaming) and a stick array that
  // fits the 256 MB cache, the y stage reads most of it from there: 256^3
  // C2C, one transform per call, fp64 y backward 93.4 -> 86.8 us (+1.2%
  // transforms/s), fp32 +2-3% (profiles/r6/mall). Batched launches (several
  // stick arrays) keep streaming: their y backward went 86 -> 107 us.
  {
    const double stickBytes = static_cast<double>(layout_.stickTotal) *
                              (floatExchange_ ? sizeof(cx<float>) : sizeof(cx<T>));
    plainHandoff_ = !distributed && !longZ_ && stickBytes <= 224.0 * (1 << 20) ? 1 : 0;
  }

  // the private stream is created on first use: a transform that runs on a
  // user stream (set_stream before its first call) never owns one
  stream_ = nullptr;
  event_.reset(new GpuEvent());

  // device tables (uploaded once; the hot path never touches the host plan)
  upload(runs_, p.runs);
  upload(runOffsets_, p.stickRunOffsets);
  if (p.simpleSticks) upload(descs_, p.stickDescs);
  zSeg_.assign(p.dimZ, 0);
  for (int r = 0; r < p.size; ++r)
    for (int z = 0; z < p.planesPerRank[r]; ++z) zSeg_[p.planeOffsets[r] + z] = r;
  std::vector<long long> sd(layout_.stickDispl.begin(), layout_.stickDispl.end());
  segStride_.assign(layout_.stickStride.begin(), layout_.stickStride.end());
  segZOff_.assign(p.planeOffsets.begin(), p.planeOffsets.end());
  upload_ztab(zTab_, sd);
  upload(colOffsets_, p.colOffsets);
  upload(colY_, p.colY);
  std::vector<long long> cb(layout_.colEntryBase.begin(), layout_.colEntryBase.end());
  upload(colBase_, cb);
  colDescs_ = true;
  build_col_desc(colDesc_, cb, layout_.slabStride);
  upload(colX_, p.colX);
  if (longX_) upload(xToCol_, p.xToCol);
  upload(twX_, make_twiddles<T>(p.dimX));
  // packed-real x stage for R2C with even dimX (SPFFT_R2C_PACKED=0 disables)
  if (!longX_ && p.type == SPFFT_TRANS_R2C && p.dimX % 2 == 0 && p.dimX >= 4 &&
      env_int("SPFFT_R2C_PACKED", 1, 0, 1) && (dev::has_ct_kernel(p.dimX / 2) ||
                                                p.dimX / 2 <= dev::max_device_fft_length(sizeof(T) == 8)))
    upload(twXh_, make_twiddles<T>(p.dimX / 2));
  upload(twY_, make_twiddles<T>(p.dimY));
  upload(twZ_, make_twiddles<T>(p.dimZ));

  batchEnabled_ = env_int("SPFFT_BATCH", 1, 0, 1) != 0;
  batchLarge_ = env_int("SPFFT_BATCH_LARGE", 1 << 22, 0, std::numeric_limits<int>::max());
  batchSplit_ = env_int("SPFFT_BATCH_SPLIT", 2, 1, dev::kMaxBatch);
  compute_batch_key();

  if (distributed) {
    const std::int64_t eb = floatExchange_ ? sizeof(cx<float>) : sizeof(cx<T>);
    for (int r = 0; r < p.size; ++r) {
      bwdSendCounts_.push_back(layout_.stickCount[r] * eb);
      bwdSendDispls_.push_back(layout_.stickDispl[r] * eb);
      bwdRecvCounts_.push_back(layout_.slabCount[r] * eb);
      bwdRecvDispls_.push_back(layout_.slabDispl[r] * eb);
    }
    // collective data-plane setup happens at plan time
    peerWrites_ = grid_->device_comm().peer_writes();
    if (peerWrites_) {
      peerStickStride_ = p.dimZ + aligned_row_pad(p.dimZ, stickElemBytes);
      if (static_cast<i64>(p.local_sticks()) * peerStickStride_ > grid_->slot_elements(GridImpl<T>::kStickSide))
        throw InvalidParameterError();
      build_peer_tables();
    }
    localDirect_ = !peerWrites_;
    if (localDirect_) {
      // this rank's own block never moves: the z stage writes it straight into
      // its place on the slab side (where the y stage and, forward, the z stage
      // read it), so the exchange skips it instead of copying it on the device
      std::vector<long long> sdl(sd);
      sdl[p.rank] = slab_offset() + layout_.slabDispl[p.rank];
      upload_ztab(zTab_, sdl);
      bwdSendCounts_[p.rank] = bwdRecvCounts_[p.rank] = 0;
    }
    // Exchange pipelining (build_chunk_plan): K plane chunks, so chunk k's
    // exchange overlaps the y/x stages of chunk k-1 (backward) or k+1
    // (forward), and I stick blocks, so block i's exchange overlaps the z stage
    // of block i+1 (backward) or i-1 (forward). Model: a step pays one grouped
    // send/recv launch (~10-20 us of fixed cost) and per-peer messages below
    // ~1.5 MB lose link efficiency, so K = per-peer bytes / 1.5 MB, between 1
    // and 4. 256^3 C2C fp64 sends 3.3 MB per peer at P = 8 (K = 2), 13 MB at
    // P = 4 and 53 MB at P = 2 (K = 4). The z stage is about a third of the
    // compute; splitting it pays only when the exchange dwarfs the step
    // overhead: I = 2 from 8 MB per peer (256^3 fp64 at P <= 4), else 1.
    // Computed from global quantities so every rank agrees;
    // SPFFT_EXCH_CHUNKS / SPFFT_EXCH_STICK_BLOCKS force the counts (rank 0's
    // values are used everywhere). The peer-write plane needs none: its stores
    // are issued by the stage kernels themselves and overlap their compute wave
    // by wave.
    const double perPeer = static_cast<double>(p.totalSticks) * p.dimZ * eb /
                           (static_cast<double>(p.size) * p.size);
    chunkModel_ = perPeer;
    int chunks = static_cast<int>(std::min(4.0, std::max(1.0, std::floor(perPeer / (1.5 * (1 << 20))))));
    chunks = env_int("SPFFT_EXCH_CHUNKS", chunks, 1, 64);
    int blocks = perPeer >= 8.0 * (1 << 20) ? 2 : 1;
    blocks = env_int("SPFFT_EXCH_STICK_BLOCKS", blocks, 1, 16);
    if (peerWrites_ || grid_->device_comm().max_pipeline_steps() == 1) chunks = blocks = 1;
    // rank 0's counts; the chunk count reduced until the (padded) layout fits
    // every rank's buffers
    int req[3] = {chunks, 1, blocks};
    while (req[1] < chunks && chunk_plan_fits(req[1] + 1)) ++req[1];
    std::vector<int> all(3 * p.size);
    grid_->communicator()->allgather(req, all.data(), sizeof(req));
    chunks = all[0];
    blocks = all[2];
    for (int r = 0; r < p.size; ++r) chunks = std::min(chunks, all[3 * r + 1]);
    if (chunks * blocks > 1 && !build_chunk_plan(chunks, blocks)) throw InternalError();
    if (!peerWrites_) register_exchanges();
  }
  log_plan();
}

// Planes that precompute (the relay plane) get every exchange of the plan
// once, here, in the same order on every rank; they then run each one without
// host round trips. Other planes return -1 and nothing is registered.
template <typename T>
void GpuExecutor<T>::register_exchanges() {
  DeviceComm& dc = grid_->device_comm();
  const IndexPlan& p = *plan_;
  if (pipelined()) {
    for (ExchangeStep& st : bwdSteps_) st.id = dc.register_exchange(GridImpl<T>::kStickSide, st.xs);
    for (ExchangeStep& st : fwdSteps_) st.id = dc.register_exchange(GridImpl<T>::kSlabSide, st.xs);
    return;
  }
  std::vector<Transfer> xs;
  append_alltoallv(xs, p.rank, p.size, bwdSendCounts_.data(), bwdSendDispls_.data(), bwdRecvCounts_.data(),
                   bwdRecvDispls_.data());
  bwdId_ = dc.register_exchange(GridImpl<T>::kStickSide, xs);
  xs.clear();
  append_alltoallv(xs, p.rank, p.size, bwdRecvCounts_.data(), bwdRecvDispls_.data(), bwdSendCounts_.data(),
                   bwdSendDispls_.data());
  fwdId_ = dc.register_exchange(GridImpl<T>::kSlabSide, xs);
}

// SPFFT_LOG=1: one line per transform with the plan decisions (engines, layout,
// data plane, pipelining)
template <typename T>
void GpuExecutor<T>::log_plan() const {
  const char* env = std::getenv("SPFFT_LOG");
  if (!env || !*env || env[0] == '0') return;
  const IndexPlan& p = *plan_;
  const bool dbl = sizeof(T) == 8;
  auto describe = [&](bool isLong, const dev::LongPlan& lp, int n, bool lf) -> std::string {
    if (!isLong) return dev::describe_engine(n, dbl, lf);
    return "long n=" + std::to_string(lp.n) + (lp.bluestein ? " bluestein m=" + std::to_string(lp.m) : "") +
           " four-step " + std::to_string(lp.n1) + "x" + std::to_string(lp.n2);
  };
  std::string plane = "none";
  if (p.size > 1) plane = const_cast<GridImpl<T>&>(*grid_).device_comm().describe();
  std::fprintf(stderr,
               "spfft[gpu rank %d/%d] %dx%dx%d %s %s: sticks=%d planes=%d columns=%d | z{%s} "
               "y{%s} x{%s}%s inter_planes=%d | exchange=%s%s plane=%s chunks=%d stick_blocks=%d "
               "steps=%zu+%zu (%.2f MB per peer) peer_writes=%d peer_offsets=[%lld, %lld] "
               "library_streams=%d\n",
               p.rank, p.size, p.dimX, p.dimY, p.dimZ,
               p.type == SPFFT_TRANS_R2C ? "R2C" : "C2C", dbl ? "fp64" : "fp32", p.local_sticks(),
               p.local_planes(), p.num_columns(),
               describe(longZ_, lpZ_, p.dimZ, false).c_str(), describe(longY_, lpY_, p.dimY, true).c_str(),
               describe(longX_, lpX_, twXh_ ? p.dimX / 2 : p.dimX, true).c_str(),
               twXh_ ? " packed-real" : "", interPlanes_, layout_.buffered ? "buffered" : "compact",
               floatExchange_ ? "-float" : "", plane.c_str(), exchChunks_, stickBlocks_, bwdSteps_.size(),
               fwdSteps_.size(), chunkModel_ / 1e6, peerWrites_ ? 1 : 0, peerOffsetRange_[0],
               peerOffsetRange_[1], GpuStream::live());
}

template <typename T>
void GpuExecutor<T>::build_col_desc(ColDescTable& t, const std::vector<long long>& colBase,
                                    long long stride) {
  const IndexPlan& p = *plan_;
  t.buf.reset();
  t.stride = stride;
  if (!colDescs_ || p.num_columns() < 1) return;
  // the kernels form y * stride in 32 bits
  if (static_cast<long long>(p.dimY) * stride >= (1LL << 31)) return;
  std::vector<dev::ColDesc> d(p.num_columns());
  for (int c = 0; c < p.num_columns(); ++c) {
    dev::ColDesc& q = d[c];
    std::vector<long long> first(dev::kColRuns, 0);
    for (int r = 0; r < dev::kColRuns; ++r) {
      q.b0[r] = 0;
      q.y[r] = 0;
      q.len[r] = 0;
    }
    int r = -1;
    for (int e = p.colOffsets[c]; e < p.colOffsets[c + 1]; ++e) {
      const bool extend = r >= 0 && p.colY[e] == q.y[r] + q.len[r] &&
                          colBase[e] == first[r] + static_cast<long long>(q.len[r]) * stride;
      if (extend) {
        ++q.len[r];
        continue;
      }
      if (++r >= dev::kColRuns) return;  // too fragmented: LDS-staged entry lists
      first[r] = colBase[e];
      q.y[r] = p.colY[e];
      q.len[r] = 1;
    }
    q.nRuns = r + 1;
    for (int k = 0; k < q.nRuns; ++k) q.b0[k] = first[k] - static_cast<long long>(q.y[k]) * stride;
  }
  upload(t.buf, d);
}

// Chunk plan of the pipelined exchange. Both exchange buffers are laid out
// chunk-major: segment v = k*P + r of the stick side holds (local sticks) x
// (chunk k of rank r's planes), block (k, q) of the slab side holds (sticks of
// rank q) x (chunk k of my planes), so chunk k is one contiguous block per peer
// on both sides. BUFFERED pads every block to maxSticks rows of
// ceil(maxPlanes / K) planes (equal counts, the reference's MPI_Alltoall
// shape); compact blocks are exact. Returns false when the padded layout does
// not fit the grid's exchange buffers (the caller tries fewer chunks).
template <typename T>
bool GpuExecutor<T>::chunk_plan_fits(int K) const {
  const IndexPlan& p = *plan_;
  if (!layout_.buffered) return true;  // compact chunks only reorder the blocks
  const i64 Mk = (static_cast<i64>(p.maxPlanes) + K - 1) / K;
  const i64 need = static_cast<i64>(K) * p.size * p.maxSticks * Mk;
  return need <= grid_->slot_elements(GridImpl<T>::kStickSide) &&
         need <= grid_->slot_elements(GridImpl<T>::kSlabSide);
}

template <typename T>
bool GpuExecutor<T>::build_chunk_plan(int K, int I) {
  const IndexPlan& p = *plan_;
  const int P = p.size, me = p.rank;
  // K and I depend on global quantities only: every rank issues the same
  // exchange steps (a rank with fewer planes or sticks gets empty ones)
  if (K < 1 || I < 1 || K * I < 2) return false;
  const bool buf = layout_.buffered;
  const i64 eb = floatExchange_ ? sizeof(cx<float>) : sizeof(cx<T>);
  auto pb = [&](int r, int k) -> i64 { return static_cast<i64>(p.planesPerRank[r]) * k / K; };
  const i64 S = p.local_sticks();
  const i64 Mk = (static_cast<i64>(p.maxPlanes) + K - 1) / K;  // padded chunk (BUFFERED)
  const i64 rowsPad = p.maxSticks;
  auto stride = [&](int r, int k) -> i64 { return buf ? Mk : pb(r, k + 1) - pb(r, k); };
  // rows of rank q's sticks on the wire, and the first row of its block i
  auto rows = [&](int q) -> i64 { return buf ? rowsPad : static_cast<i64>(p.sticksPerRank[q]); };
  auto rb = [&](int q, int i) -> i64 { return rows(q) * i / I; };
  const int NV = K * P;
  std::vector<long long> segDispl(NV), segStride(NV);
  std::vector<int> segZOff(NV), zSeg(p.dimZ, 0);
  i64 off = 0;
  for (int k = 0; k < K; ++k) {
    for (int r = 0; r < P; ++r) {
      const int v = k * P + r;
      const i64 n = pb(r, k + 1) - pb(r, k);
      segDispl[v] = off;
      segStride[v] = stride(r, k);
      segZOff[v] = p.planeOffsets[r] + static_cast<int>(pb(r, k));
      for (i64 z = 0; z < n; ++z) zSeg[segZOff[v] + z] = v;
      off += rows(me) * segStride[v];
    }
  }
  if (off > grid_->slot_elements(GridImpl<T>::kStickSide)) return false;
  std::vector<i64> slabDispl(NV);
  i64 soff = 0;
  for (int k = 0; k < K; ++k) {
    for (int q = 0; q < P; ++q) {
      slabDispl[k * P + q] = soff;
      soff += rows(q) * stride(me, k);
    }
  }
  if (soff > grid_->slot_elements(GridImpl<T>::kSlabSide)) return false;
  if (!buf && (off != layout_.stickTotal || soff != layout_.slabTotal)) throw InternalError();
  planeBounds_.resize(K + 1);
  for (int k = 0; k <= K; ++k) planeBounds_[k] = static_cast<int>(pb(me, k));
  // z launch i covers the sticks of message rows [rb(me, i), rb(me, i + 1))
  stickBounds_.resize(I + 1);
  for (int i = 0; i <= I; ++i) stickBounds_[i] = static_cast<int>(std::min(S, rb(me, i)));
  colBaseChunk_.clear();
  colDescChunk_.clear();
  for (int k = 0; k < K; ++k) {
    const i64 sk = stride(me, k);
    // entry e at local plane z of chunk k: base + z (z in [pb_k, pb_k+1))
    std::vector<long long> cb(p.colY.size());
    for (std::size_t e = 0; e < p.colY.size(); ++e)
      cb[e] = slabDispl[k * P + p.colRank[e]] + static_cast<i64>(p.colLocal[e]) * sk - pb(me, k);
    colBaseChunk_.emplace_back();
    upload(colBaseChunk_.back(), cb);
    colDescChunk_.emplace_back();
    build_col_desc(colDescChunk_.back(), cb, sk);
  }
  // transfer list of message (i, k) in the backward direction
  auto cell = [&](int i, int k, std::vector<Transfer>& out) {
    std::vector<std::int64_t> sc(P), sd(P), rc(P), rd(P);
    for (int r = 0; r < P; ++r) {
      const int v = k * P + r;
      sd[r] = (segDispl[v] + rb(me, i) * segStride[v]) * eb;
      sc[r] = (rb(me, i + 1) - rb(me, i)) * segStride[v] * eb;
      rd[r] = (slabDispl[v] + rb(r, i) * stride(me, k)) * eb;
      rc[r] = (rb(r, i + 1) - rb(r, i)) * stride(me, k) * eb;
    }
    if (localDirect_) sc[me] = rc[me] = 0;  // own block in place on the slab side
    append_alltoallv(out, me, P, sc.data(), sd.data(), rc.data(), rd.data());
  };
  // backward: blocks 0..I-2 as soon as their z launch is done, each with every
  // chunk; the last block chunk by chunk, chunk k's arrival releases y/x(k)
  bwdSteps_.clear();
  for (int i = 0; i + 1 < I; ++i) {
    ExchangeStep st{{}, 1, i, 0, 0};
    for (int k = 0; k < K; ++k) cell(i, k, st.xs);
    bwdSteps_.push_back(std::move(st));
  }
  for (int k = 0; k < K; ++k) {
    ExchangeStep st{{}, k == 0 ? 1 : 0, I - 1, 2, k};
    cell(I - 1, k, st.xs);
    bwdSteps_.push_back(std::move(st));
  }
  // forward (send and receive roles swapped): chunks 0..K-2 as soon as their y
  // stage is done, each with every block; the last chunk block by block, block
  // i's arrival releases z(i)
  auto mirror = [](std::vector<Transfer>& xs) {
    for (Transfer& t : xs) {
      if (t.kind == Transfer::kLocal)
        std::swap(t.offset, t.dstOffset);
      else
        t.kind = t.kind == Transfer::kSend ? Transfer::kRecv : Transfer::kSend;
    }
    // a receive from q mirrors into a send to q: the staggered order of the
    // backward list (send me+k, receive me-k) becomes (receive me+k, send
    // me-k), which pairs across ranks in the same order
  };
  fwdSteps_.clear();
  for (int k = 0; k + 1 < K; ++k) {
    ExchangeStep st{{}, 2, k, 0, 0};
    for (int i = 0; i < I; ++i) cell(i, k, st.xs);
    mirror(st.xs);
    fwdSteps_.push_back(std::move(st));
  }
  for (int i = 0; i < I; ++i) {
    ExchangeStep st{{}, i == 0 ? 2 : 0, K - 1, 3, i};
    cell(i, K - 1, st.xs);
    mirror(st.xs);
    fwdSteps_.push_back(std::move(st));
  }
  if (localDirect_)
    for (int k = 0; k < K; ++k) segDispl[k * P + me] = slab_offset() + slabDispl[k * P + me];
  zSeg_ = zSeg;
  segStride_ = segStride;
  segZOff_ = segZOff;
  upload_ztab(zTab_, segDispl);
  exchChunks_ = K;
  stickBlocks_ = I;
  auto events = [](std::vector<std::unique_ptr<GpuEvent>>& v, int n) {
    v.clear();
    for (int j = 0; j < n; ++j) v.emplace_back(new GpuEvent());
  };
  events(zEv_, I);
  events(blockEv_, I);
  events(chunkEv_, K);
  return true;
}

// Device table of the z stage's exchange segments: per plane z its segment's
// (segDispl - segZOff + z, segStride), so (stick s, plane z) is one entry away.
template <typename T>
void GpuExecutor<T>::upload_ztab(std::unique_ptr<DeviceBuffer>& dst,
                                 const std::vector<long long>& segDispl) {
  const int Z = plan_->dimZ;
  std::vector<long long> tab(2 * static_cast<std::size_t>(Z));
  for (int z = 0; z < Z; ++z) {
    const int v = zSeg_[z];
    tab[2 * z] = segDispl[v] - segZOff_[v] + z;
    tab[2 * z + 1] = segStride_[v];
  }
  upload(dst, tab);
}

// Element offset (exchange element type) from the stick-side buffer to the
// slab-side buffer of this rank's grid.
template <typename T>
long long GpuExecutor<T>::slab_offset() const {
  const i64 eb = floatExchange_ ? sizeof(cx<float>) : sizeof(cx<T>);
  const char* stick = static_cast<const char*>(grid_->device_slot(GridImpl<T>::kStickSide));
  const char* slab = static_cast<const char*>(grid_->device_slot(GridImpl<T>::kSlabSide));
  const long long d = slab - stick;
  if (d % eb != 0) throw InternalError();
  return d / eb;
}

template <typename T>
hipEvent_t GpuExecutor<T>::step_event(int kind, int idx) const {
  switch (kind) {
    case 1:
      return zEv_[idx]->get();
    case 2:
      return chunkEv_[idx]->get();
    case 3:
      return blockEv_[idx]->get();
    default:
      return nullptr;
  }
}

template <typename T>
void GpuExecutor<T>::run_steps(const std::vector<ExchangeStep>& steps, bool backward) {
  DeviceGuard guard(deviceId_);
  void* stick = grid_->device_slot(GridImpl<T>::kStickSide);
  void* slab = grid_->device_slot(GridImpl<T>::kSlabSide);
  DeviceComm& dc = grid_->device_comm();
  // SPFFT_TIMING: the span from the first step's start to the last step's
  // completion on the data plane's stream (gpu/<direction>/exchange-span)
  GpuEvent *b = nullptr, *e = nullptr;
  if (timing::gpu_stages() && !capturing_ && !steps.empty()) {
    spans_.push_back(ExchangeSpan{backward ? "backward" : "forward", timing_event(), timing_event()});
    b = spans_.back().begin.get();
    e = spans_.back().end.get();
  }
  for (std::size_t j = 0; j < steps.size(); ++j) {
    const ExchangeStep& st = steps[j];
    const ExchangeSync sync{step_event(st.readyKind, st.readyIdx), step_event(st.doneKind, st.doneIdx),
                            j == 0 && b ? b->get() : nullptr,
                            j + 1 == steps.size() && e ? e->get() : nullptr};
    if (st.id >= 0)
      dc.exchange_registered(st.id, stream_, &sync);
    else if (backward)
      dc.exchange(stick, slab, st.xs, stream_, &sync);
    else
      dc.exchange(slab, stick, st.xs, stream_, &sync);
  }
}

template <typename T>
void GpuExecutor<T>::pipelined_exchange(bool backward) {
  // backward: z(i) recorded zEv_[i] (backward_z); y/x(k) wait for chunkEv_[k]
  // (backward_xy). forward: y(k) recorded chunkEv_[k] (forward_xy); z(i) waits
  // for blockEv_[i] (forward_z)
  run_steps(backward ? bwdSteps_ : fwdSteps_, backward);
}

template <typename T>
void GpuExecutor<T>::build_peer_tables() {
  const IndexPlan& p = *plan_;
  DeviceComm& dc = grid_->device_comm();
  const int P = p.size, me = p.rank;
  const i64 eb = floatExchange_ ? sizeof(cx<float>) : sizeof(cx<T>);
  const char* stick = static_cast<const char*>(grid_->device_slot(GridImpl<T>::kStickSide));
  const char* slab = static_cast<const char*>(grid_->device_slot(GridImpl<T>::kSlabSide));
  auto elem_offset = [&](const void* peer, const char* local) -> long long {
    if (!peer) throw InternalError();
    const long long d = static_cast<const char*>(peer) - local;
    if (d % eb != 0) throw InternalError();
    return d / eb;
  };
  const i64 block = static_cast<i64>(p.maxSticks) * p.maxPlanes;
  i64 sticksBefore = 0, planesBefore = 0;
  for (int q = 0; q < me; ++q) {
    sticksBefore += p.sticksPerRank[q];
    planesBefore += p.planesPerRank[q];
  }
  // backward: my sticks' planes of rank r land in r's slab side, block "from me"
  std::vector<long long> seg(P);
  for (int r = 0; r < P; ++r) {
    const i64 displ = layout_.buffered ? me * block : sticksBefore * p.planesPerRank[r];
    seg[r] = elem_offset(dc.peer_buffer(r, GridImpl<T>::kSlabSide), stick) + displ;
  }
  upload_ztab(zTabRemote_, seg);  // peer writes never chunk: per-rank segments
  // forward: column entries of rank r's sticks land in r's stick side, which
  // peer writes keep in the single-rank layout (stick s, plane z at
  // s * peerStickStride_ + z, every rank's planes in place): no exchange block
  // has to be contiguous, so the z forward stage reads plain stick rows (no
  // per-plane segment table: 2 ranks on one GPU, 256^3, z forward 124 -> 57
  // us per rank, 3546 -> 3851 transforms/s; profiles/r6/shared_gpu)
  std::vector<long long> cb(p.colY.size());
  std::vector<long long> base(P);
  for (int r = 0; r < P; ++r)
    base[r] = elem_offset(dc.peer_buffer(r, GridImpl<T>::kStickSide), slab) + planesBefore;
  for (std::size_t k = 0; k < p.colY.size(); ++k)
    cb[k] = base[p.colRank[k]] + static_cast<i64>(p.colLocal[k]) * peerStickStride_;
  upload(colBaseRemote_, cb);
  build_col_desc(colDescRemote_, cb, peerStickStride_);
  // peers' buffers are addressed as element offsets from the local ones: both
  // signs occur (the descriptor and list paths take signed 64-bit bases)
  peerOffsetRange_[0] = peerOffsetRange_[1] = 0;
  for (long long v : seg) {
    peerOffsetRange_[0] = std::min(peerOffsetRange_[0], v);
    peerOffsetRange_[1] = std::max(peerOffsetRange_[1], v);
  }
  for (long long v : base) {
    peerOffsetRange_[0] = std::min(peerOffsetRange_[0], v);
    peerOffsetRange_[1] = std::max(peerOffsetRange_[1], v);
  }
}

template <typename T>
GpuExecutor<T>::~GpuExecutor() {
  if (process_exiting()) return;
  try {
    DeviceGuard guard(deviceId_);
    if (stream_) (void)hipStreamSynchronize(stream_);
    for (auto& g : graphs_) (void)hipGraphExecDestroy(g.exec);
  } catch (...) {
  }
}

template <typename T>
void GpuExecutor<T>::set_stream(hipStream_t stream, bool synchronous) {
  stream_ = stream;
  ownStreamActive_ = false;
  synchronous_ = synchronous;
}

template <typename T>
void GpuExecutor<T>::reset_stream() {
  ownStreamActive_ = true;
  synchronous_ = true;
  stream_ = nullptr;
  use_private_stream();
}

template <typename T>
void GpuExecutor<T>::use_private_stream() {
  if (!ownStreamActive_ || stream_) return;
  DeviceGuard guard(deviceId_);
  if (!ownStream_) ownStream_.reset(new GpuStream());
  stream_ = ownStream_->get();
}

template <typename T>
void GpuExecutor<T>::synchronize() {
  wait_stream();
  if (!traces_.empty() || !spans_.empty()) harvest_stage_times(false);
  // a peer barrier that timed out leaves a flag behind (data are incomplete)
  if (peerWrites_) grid_->device_comm().check();
}

template <typename T>
void GpuExecutor<T>::wait_stream() {
  DeviceGuard guard(deviceId_);
  if (plan_->size > 1) {
    wait_stream_watched();
    return;
  }
  if (gpu_sync_spin()) {
    // poll: wakes within ~1 us of completion instead of the blocking wait's
    // interrupt latency; falls back to the blocking wait after ~20 ms
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipStreamQuery(stream_);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) gpu_check(e, "hipStreamQuery");
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
    }
  }
  gpu_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

// ---------------------------------------------------------- stage timing
template <typename T>
void GpuExecutor<T>::stage_mark(const char* dir, const char* stage) {
  if (!timing::gpu_stages() || capturing_) return;
  if (!stage) {
    // a direction starts: collect what has completed, bound the backlog
    harvest_stage_times(traces_.size() >= 64);
    traces_.push_back(StageTrace{dir, {}});
  }
  if (traces_.empty() || traces_.back().dir != dir) return;
  StageMark m;
  m.ev = timing_event();
  m.ev->record(stream_);
  m.stage = stage;
  traces_.back().marks.push_back(std::move(m));
}

template <typename T>
std::unique_ptr<GpuEvent> GpuExecutor<T>::timing_event() {
  if (spareEvents_.empty()) return std::unique_ptr<GpuEvent>(new GpuEvent(true));
  std::unique_ptr<GpuEvent> ev = std::move(spareEvents_.back());
  spareEvents_.pop_back();
  return ev;
}

template <typename T>
void GpuExecutor<T>::harvest_stage_times(bool wait) {
  std::size_t spansDone = 0;
  for (auto& sp : spans_) {
    if (wait) {
      gpu_check(hipEventSynchronize(sp.end->get()), "hipEventSynchronize");
    } else {
      const hipError_t e = hipEventQuery(sp.end->get());
      if (e == hipErrorNotReady) break;
      gpu_check(e, "hipEventQuery");
    }
    float ms = 0;
    if (hipEventElapsedTime(&ms, sp.begin->get(), sp.end->get()) == hipSuccess)
      timing::add_sample({"gpu", sp.dir, "exchange-span"}, 1e-3 * ms);
    spareEvents_.push_back(std::move(sp.begin));
    spareEvents_.push_back(std::move(sp.end));
    ++spansDone;
  }
  spans_.erase(spans_.begin(), spans_.begin() + static_cast<std::ptrdiff_t>(spansDone));
  std::size_t done = 0;
  for (auto& t : traces_) {
    if (t.marks.empty()) {
      ++done;
      continue;
    }
    hipEvent_t last = t.marks.back().ev->get();
    if (wait) {
      gpu_check(hipEventSynchronize(last), "hipEventSynchronize");
    } else {
      const hipError_t e = hipEventQuery(last);
      if (e == hipErrorNotReady) break;
      gpu_check(e, "hipEventQuery");
    }
    for (std::size_t i = 1; i < t.marks.size(); ++i) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, t.marks[i - 1].ev->get(), t.marks[i].ev->get()) == hipSuccess)
        timing::add_sample({"gpu", t.dir, t.marks[i].stage}, 1e-3 * ms);
    }
    for (auto& m : t.marks) spareEvents_.push_back(std::move(m.ev));
    ++done;
  }
  traces_.erase(traces_.begin(), traces_.begin() + static_cast<std::ptrdiff_t>(done));
  (void)hipGetLastError();
}

// Failure detection for distributed transforms: the
// host polls the stream and, every millisecond, the data plane's asynchronous
// error state (RCCL: ncclCommGetAsyncError; peer writes: barrier timeouts). A
// failure, or a wait longer than SPFFT_COMM_TIMEOUT seconds (default 0 = no
// limit), aborts the data plane (ncclCommAbort / barrier kernels released)
// and throws MPIError with the cause in the error detail, instead of leaving
// the caller blocked forever on a dead peer.
template <typename T>
void GpuExecutor<T>::wait_stream_watched() {
  DeviceComm& dc = grid_->device_comm();
  const double timeout = comm_timeout_seconds();
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  auto last = t0;
  for (;;) {
    const hipError_t e = hipStreamQuery(stream_);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) gpu_check(e, "hipStreamQuery");
    const auto now = clock::now();
    if (now - last >= std::chrono::milliseconds(1)) {
      last = now;
      std::string detail;
      const double waited = std::chrono::duration<double>(now - t0).count();
      if (dc.healthy(&detail) && timeout > 0 && waited > timeout)
        detail = "exchange did not complete within SPFFT_COMM_TIMEOUT = " + std::to_string(timeout) +
                 " s";
      if (!detail.empty()) {
        dc.abort();
        set_error_detail(detail + " (data plane aborted)");
        throw MPIError();
      }
    }
    // spin for the first ~20 ms (low wake-up latency), then yield the core
    if (now - t0 > std::chrono::milliseconds(20)) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// ------------------------------------------------------------- graph replay
template <typename T>
bool GpuExecutor<T>::graph_eligible() const {
  // single rank only: exchanges (RCCL, peer barriers) stay outside graphs; the
  // legacy default stream cannot be captured
  return graphsEnabled_ && plan_->size == 1 && !poison_ && !gpu_sync_debug() &&
         stream_ != nullptr;
}

template <typename T>
template <class Enqueue>
bool GpuExecutor<T>::replay(const GraphEntry& key, Enqueue enqueue) {
  DeviceGuard guard(deviceId_);
  GraphEntry* hit = nullptr;
  for (auto& g : graphs_)
    if (g.dir == key.dir && g.in == key.in && g.out == key.out && g.scaling == key.scaling &&
        g.stream == key.stream)
      hit = &g;
  if (!hit) {
    if (!warm_[key.dir]) {
      // the first call of a direction runs eagerly (kernel attributes, lazy
      // module loading happen outside any capture)
      warm_[key.dir] = true;
      return false;
    }
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    bool ok = hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal) == hipSuccess;
    if (ok) {
      capturing_ = true;
      try {
        enqueue();
      } catch (...) {
        ok = false;
      }
      capturing_ = false;
      ok = hipStreamEndCapture(stream_, &graph) == hipSuccess && ok && graph;
      if (ok) ok = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess;
      if (graph) (void)hipGraphDestroy(graph);
    }
    if (!ok) {
      // capture unsupported here: run step-wise from now on
      (void)hipGetLastError();
      graphsEnabled_ = false;
      if (exec) (void)hipGraphExecDestroy(exec);
      return false;
    }
    if (graphs_.size() >= 8) {
      (void)hipGraphExecDestroy(graphs_.front().exec);
      graphs_.erase(graphs_.begin());
    }
    GraphEntry e = key;
    e.exec = exec;
    graphs_.push_back(e);
    hit = &graphs_.back();
  }
  order_after_default_stream();
  gpu_check(hipGraphLaunch(hit->exec, stream_), "hipGraphLaunch");
  return true;
}

template <typename T>
bool GpuExecutor<T>::backward_graph(const T* input, SpfftProcessingUnitType outputLocation) {
  if (!graph_eligible() || outputLocation != SPFFT_PU_GPU) return false;
  const bool any = plan_->numLocalElements > 0;
  if (any && (!input || !is_device_pointer(input))) return false;
  if (hipGetLastError() != hipSuccess) throw GPUPrecedingError();
  SPFFT_TIMED_SCOPE("gpu_backward_graph");
  const GraphEntry key{0, any ? input : nullptr, nullptr, 0, stream_, nullptr};
  return replay(key, [&] {
    backward_z(input);
    backward_xy(SPFFT_PU_GPU);
  });
}

template <typename T>
bool GpuExecutor<T>::forward_graph(SpfftProcessingUnitType inputLocation, T* output,
                                   SpfftScalingType scaling) {
  if (!graph_eligible() || inputLocation != SPFFT_PU_GPU) return false;
  const bool any = plan_->numLocalElements > 0;
  if (any && (!output || !is_device_pointer(output))) return false;
  if (hipGetLastError() != hipSuccess) throw GPUPrecedingError();
  SPFFT_TIMED_SCOPE("gpu_forward_graph");
  const GraphEntry key{1, nullptr, any ? output : nullptr, static_cast<int>(scaling), stream_, nullptr};
  return replay(key, [&] {
    forward_xy(SPFFT_PU_GPU);
    forward_z(output, scaling);
  });
}

template <typename T>
void GpuExecutor<T>::order_after_default_stream() {
  use_private_stream();
  if (capturing_) return;
  // errors left behind by earlier (user) GPU work (reference: execution_gpu.cpp:251-253)
  if (hipGetLastError() != hipSuccess) throw GPUPrecedingError();
  if (ownStreamActive_) {
    // order after work already queued on the legacy default stream (reference: execution_gpu.cpp:258-259)
    event_->record(nullptr);
    event_->wait_on(stream_);
  }
}

template <typename T>
cx<T>* GpuExecutor<T>::staging(std::size_t elems) {
  const std::size_t bytes = std::max<std::size_t>(1, elems) * sizeof(cx<T>);
  if (!staging_ || staging_->bytes() < bytes) staging_.reset(new DeviceBuffer(bytes));
  return staging_->data<cx<T>>();
}

template <typename T>
std::size_t GpuExecutor<T>::space_bytes() const {
  const IndexPlan& p = *plan_;
  const std::size_t elems = static_cast<std::size_t>(p.local_planes()) * p.dimY * p.dimX;
  return elems * (p.type == SPFFT_TRANS_R2C ? sizeof(T) : sizeof(cx<T>));
}

template <typename T>
T* GpuExecutor<T>::space_domain(SpfftProcessingUnitType location) {
  if (location == SPFFT_PU_GPU) return static_cast<T*>(grid_->device_slot(GridImpl<T>::kSpace));
  if (location == SPFFT_PU_HOST) return static_cast<T*>(grid_->host_slot(GridImpl<T>::kSpace));
  throw InvalidParameterError();
}

template <typename T>
dev::ZArgs GpuExecutor<T>::zargs() const {
  const IndexPlan& p = *plan_;
  dev::ZArgs a{};
  a.numSticks = p.local_sticks();
  a.stickBegin = 0;
  a.n = p.dimZ;
  a.zeroStick = p.type == SPFFT_TRANS_R2C ? p.zeroStick : -1;
  a.runs = runs_ ? runs_->data<StickRun>() : nullptr;
  a.runOffsets = runOffsets_ ? runOffsets_->data<int>() : nullptr;
  a.desc = descs_ ? descs_->data<StickDesc>() : nullptr;
  a.single = p.size == 1 ? 1 : 0;
  a.stickStride = layout_.stickStride[0];
  a.zTab = zTab_ ? zTab_->data<long long>() : nullptr;
  // Forward value stores streamed when one transform's values outgrow what the
  // 256 MB Infinity Cache keeps: 512^3 R2C fp32 (282 MB of values) T = 4 1870
  // -> 1900 transforms/s; 256^3 (70 / 140 MB) kept plain, nt there lost 2-3%
  // (profiles/r6/ntmerge/zf_values_ab.txt)
  a.ntValueStores = static_cast<double>(p.numLocalElements) * sizeof(cx<T>) > 192.0 * (1 << 20) ? 1 : 0;
  return a;
}

template <typename T>
dev::YArgs GpuExecutor<T>::yargs() const {
  const IndexPlan& p = *plan_;
  dev::YArgs a{};
  a.ncols = p.num_columns();
  a.colBegin = 0;
  a.colEnd = a.ncols;
  a.L = p.local_planes();
  a.zBegin = 0;
  a.n = p.dimY;
  a.colOfX0 = p.type == SPFFT_TRANS_R2C ? p.colOfX0 : -1;
  a.interStride = interStride_;
  a.interZStride = static_cast<long long>(p.num_columns()) * interStride_;
  a.colOffsets = colOffsets_ ? colOffsets_->data<int>() : nullptr;
  a.colY = colY_ ? colY_->data<int>() : nullptr;
  a.colBase = colBase_ ? colBase_->data<long long>() : nullptr;
  set_col_desc(a, colDesc_);
  return a;
}

template <typename T>
dev::XArgs GpuExecutor<T>::xargs() const {
  const IndexPlan& p = *plan_;
  dev::XArgs a{};
  a.L = p.local_planes();
  a.zBegin = 0;
  a.Y = p.dimY;
  a.n = p.dimX;
  a.nFreq = p.dimXFreq;
  a.ncols = p.num_columns();
  a.interStride = interStride_;
  a.interZStride = static_cast<long long>(p.num_columns()) * interStride_;
  a.colX = colX_ ? colX_->data<int>() : nullptr;
  a.xToCol = xToCol_ ? xToCol_->data<int>() : nullptr;
  return a;
}

// NaN poisoning (debug aid, generalises the reference tests' "run twice"):
// every work buffer a direction writes before reading is filled with NaN bytes
// first, so a kernel that reads an element nobody wrote shows up as NaN output.
template <typename T>
void GpuExecutor<T>::poison(bool backward) {
  if (!poison_ || capturing_) return;
  auto fill = [&](typename GridImpl<T>::Slot slot) {
    gpu_check(hipMemsetAsync(grid_->device_slot(slot), 0xFF,
                             static_cast<std::size_t>(grid_->device_slot_elements(slot)) * sizeof(cx<T>),
                             stream_),
              "hipMemsetAsync");
  };
  fill(GridImpl<T>::kInter);
  if (backward) {
    fill(GridImpl<T>::kSpace);
    if (plan_->size == 1 || !peerWrites_) fill(GridImpl<T>::kStickSide);
    if (plan_->size == 1) fill(GridImpl<T>::kSlabSide);
  } else if (plan_->size == 1) {
    fill(GridImpl<T>::kStickSide);
    fill(GridImpl<T>::kSlabSide);
  }
}

// ------------------------------------------------------------------ backward
template <typename T>
void GpuExecutor<T>::backward_z(const T* input) {
  SPFFT_TIMED_SCOPE("gpu_backward_z");
  DeviceGuard guard(deviceId_);
  order_after_default_stream();
  stage_mark("backward", nullptr);
  StageEnd stageEnd{this, "backward", "z"};
  poison(true);
  const IndexPlan& p = *plan_;
  const cx<T>* values = reinterpret_cast<const cx<T>*>(input);
  if (p.numLocalElements > 0) {
    if (!input) throw InvalidParameterError();
    // (a capture only runs for device-resident input: backward_graph)
    if (!capturing_ && !is_device_pointer(input)) {
      cx<T>* st = staging(p.numLocalElements);
      gpu_check(hipMemcpyAsync(st, input, sizeof(cx<T>) * p.numLocalElements,
                               hipMemcpyHostToDevice, stream_),
                "hipMemcpyAsync");
      values = st;
    }
  }
  void* stick = grid_->device_slot(GridImpl<T>::kStickSide);
  auto a = zargs();
  a.plainSticks = plainHandoff_;
  if (peerWrites_) {
    // the z stage stores straight into the peers' slab sides
    grid_->device_comm().prepare_write(GridImpl<T>::kSlabSide, stream_);
    a.zTab = zTabRemote_->data<long long>();
    // (no fence in the kernel: the barrier round after it writes back every
    // XCD's L2, peer_sync.hip)
  }
  // pipelined plans: one launch per stick block, whose messages leave as soon
  // as it is done (zEv_, run_steps)
  const int I = pipelined() ? stickBlocks_ : 1;
  for (int i = 0; i < I; ++i) {
    if (pipelined()) {
      a.stickBegin = stickBounds_[i];
      a.numSticks = stickBounds_[i + 1];
    }
    z_backward_launch(a, values, stick);
    if (pipelined()) zEv_[i]->record(stream_);
  }
}

template <typename T>
void GpuExecutor<T>::z_backward_launch(const dev::ZArgs& a, const cx<T>* values, void* stick) {
  if (longZ_ && floatExchange_)
    dev::launch_long_z_backward<T, cx<float>>(lpZ_, a, values, static_cast<cx<float>*>(stick),
                                              long_bufs(), stream_);
  else if (longZ_)
    dev::launch_long_z_backward<T, cx<T>>(lpZ_, a, values, static_cast<cx<T>*>(stick), long_bufs(),
                                          stream_);
  else if (floatExchange_)
    dev::launch_z_backward<T, cx<float>>(a, values, static_cast<cx<float>*>(stick),
                                         twZ_->data<cx<T>>(), stream_);
  else
    dev::launch_z_backward<T, cx<T>>(a, values, static_cast<cx<T>*>(stick), twZ_->data<cx<T>>(),
                                     stream_);
}

template <typename T>
void GpuExecutor<T>::exchange(bool backward) {
  if (plan_->size <= 1) return;
  DeviceGuard guard(deviceId_);
  void* stick = grid_->device_slot(GridImpl<T>::kStickSide);
  void* slab = grid_->device_slot(GridImpl<T>::kSlabSide);
  DeviceComm& dc = grid_->device_comm();
  const int id = backward ? bwdId_ : fwdId_;
  if (id >= 0)
    dc.exchange_registered(id, stream_, nullptr);
  else if (backward)
    dc.alltoallv(stick, bwdSendCounts_.data(), bwdSendDispls_.data(), slab, bwdRecvCounts_.data(),
                 bwdRecvDispls_.data(), stream_);
  else
    dc.alltoallv(slab, bwdRecvCounts_.data(), bwdRecvDispls_.data(), stick, bwdSendCounts_.data(),
                 bwdSendDispls_.data(), stream_);
}

template <typename T>
void GpuExecutor<T>::backward_exchange(bool /*nonBlocking*/) {
  SPFFT_TIMED_SCOPE("gpu_backward_exchange");
  // pipelined: the exchange runs on the comm stream, inside "exchange+y+x"
  StageEnd stageEnd{this, "backward", pipelined() ? nullptr : "exchange"};
  if (peerWrites_) {
    DeviceGuard guard(deviceId_);
    grid_->device_comm().complete_writes(stream_);
    return;
  }
  if (pipelined()) {
    pipelined_exchange(true);
    return;
  }
  exchange(true);
}

// ------------------------------------------------------------- long axes
// Axes longer than one workgroup's LDS (or with a large prime factor and no
// in-LDS Bluestein, or line-fast axes whose run-time engine would hold less than
// a column segment) run the global four-step / Bluestein FFT with the stage IO
// fused into its passes (kernels/long_fft.hpp: needs_long_path).
template <typename T>
void GpuExecutor<T>::setup_long_axes() {
  const IndexPlan& p = *plan_;
  const bool dbl = sizeof(T) == 8;
  const bool packedX = p.type == SPFFT_TRANS_R2C && p.dimX % 2 == 0 && p.dimX >= 4;
  const int xLen = packedX ? p.dimX / 2 : p.dimX;
  longZ_ = dev::needs_long_path(p.dimZ, dbl, dev::kLongAxisZ);
  longY_ = dev::needs_long_path(p.dimY, dbl, dev::kLongAxisY);
  longX_ = dev::needs_long_path(xLen, dbl, dev::kLongAxisX);
  long long elems = 0;
  if (longZ_) {
    lpZ_ = dev::long_plan(p.dimZ, dbl);
    elems = std::max(elems, static_cast<long long>(p.local_sticks()) * (lpZ_.line_elems() + 2));
  }
  if (longY_) {
    lpY_ = dev::long_plan(p.dimY, dbl);
    elems = std::max(elems, static_cast<long long>(interPlanes_) * p.num_columns() *
                                (lpY_.line_elems() + 2));
  }
  if (longX_) {
    lpX_ = dev::long_plan(xLen, dbl);
    elems = std::max(elems, static_cast<long long>(interPlanes_) * p.dimY *
                                (std::max<long long>(lpX_.line_elems(), p.dimX) + 2));
  }
  if (elems == 0) return;
  const bool blue = (longZ_ && lpZ_.bluestein) || (longY_ && lpY_.bluestein) ||
                    (longX_ && lpX_.bluestein);
  const std::size_t bytes = static_cast<std::size_t>(elems) * sizeof(cx<T>);
  for (int i = 0; i < 4; ++i)
    if (blue || i == 0 || i == 3) longWork_[i].reset(new DeviceBuffer(bytes));
}

template <typename T>
dev::LongBufs<T> GpuExecutor<T>::long_bufs() const {
  auto ptr = [&](int i) { return longWork_[i] ? longWork_[i]->template data<cx<T>>() : nullptr; };
  return dev::LongBufs<T>{ptr(0), ptr(1), ptr(2), ptr(3)};
}

template <typename T>
void GpuExecutor<T>::y_backward_launch(const dev::YArgs& ya, const void* slab, cx<T>* inter) {
  if (longY_ && floatExchange_)
    dev::launch_long_y_backward<T, cx<float>>(lpY_, ya, static_cast<const cx<float>*>(slab), inter,
                                              long_bufs(), stream_);
  else if (longY_)
    dev::launch_long_y_backward<T, cx<T>>(lpY_, ya, static_cast<const cx<T>*>(slab), inter,
                                          long_bufs(), stream_);
  else if (floatExchange_)
    dev::launch_y_backward<T, cx<float>>(ya, static_cast<const cx<float>*>(slab), inter,
                                         twY_->data<cx<T>>(), stream_);
  else
    dev::launch_y_backward<T, cx<T>>(ya, static_cast<const cx<T>*>(slab), inter, twY_->data<cx<T>>(),
                                     stream_);
}

template <typename T>
void GpuExecutor<T>::y_forward_launch(const dev::YArgs& ya, cx<T>* inter, void* slab) {
  if (longY_ && floatExchange_)
    dev::launch_long_y_forward<T, cx<float>>(lpY_, ya, inter, static_cast<cx<float>*>(slab),
                                             long_bufs(), stream_);
  else if (longY_)
    dev::launch_long_y_forward<T, cx<T>>(lpY_, ya, inter, static_cast<cx<T>*>(slab), long_bufs(),
                                         stream_);
  else if (floatExchange_)
    dev::launch_y_forward<T, cx<float>>(ya, inter, static_cast<cx<float>*>(slab), twY_->data<cx<T>>(),
                                        stream_);
  else
    dev::launch_y_forward<T, cx<T>>(ya, inter, static_cast<cx<T>*>(slab), twY_->data<cx<T>>(), stream_);
}

template <typename T>
void GpuExecutor<T>::x_backward_launch(const dev::XArgs& xa, const cx<T>* inter, void* space) {
  const bool r2c = plan_->type == SPFFT_TRANS_R2C;
  if (longX_)
    dev::launch_long_x_backward<T>(lpX_, xa, r2c, inter, space, twX_->data<cx<T>>(), long_bufs(),
                                   stream_);
  else
    dev::launch_x_backward<T>(xa, r2c, inter, space, twX_->data<cx<T>>(),
                              twXh_ ? twXh_->data<cx<T>>() : nullptr, stream_);
}

template <typename T>
void GpuExecutor<T>::x_forward_launch(const dev::XArgs& xa, const void* space, cx<T>* inter) {
  const bool r2c = plan_->type == SPFFT_TRANS_R2C;
  if (longX_)
    dev::launch_long_x_forward<T>(lpX_, xa, r2c, space, inter, twX_->data<cx<T>>(), long_bufs(),
                                  stream_);
  else
    dev::launch_x_forward<T>(xa, r2c, space, inter, twX_->data<cx<T>>(),
                             twXh_ ? twXh_->data<cx<T>>() : nullptr, stream_);
}

// The intermediate as seen by the y/x kernels of a plane range starting at z0:
// they address plane z at z * interZStride, so a capped buffer is shifted to
// hold planes [z0, z0 + interPlanes_).
template <typename T>
cx<T>* GpuExecutor<T>::inter_for(cx<T>* inter, int z0) const {
  if (interPlanes_ >= plan_->local_planes()) return inter;
  return inter - static_cast<long long>(z0) * plan_->num_columns() * interStride_;
}

template <typename T>
void GpuExecutor<T>::backward_xy(SpfftProcessingUnitType outputLocation) {
  SPFFT_TIMED_SCOPE("gpu_backward_xy");
  if (outputLocation != SPFFT_PU_HOST && outputLocation != SPFFT_PU_GPU)
    throw InvalidParameterError();
  DeviceGuard guard(deviceId_);
  StageEnd stageEnd{this, "backward", pipelined() ? "exchange+y+x" : "y+x"};
  void* slab = grid_->device_slot(GridImpl<T>::kSlabSide);
  auto* inter = static_cast<cx<T>*>(grid_->device_slot(GridImpl<T>::kInter));
  void* space = grid_->device_slot(GridImpl<T>::kSpace);
  if (peerWrites_) grid_->device_comm().note_read(GridImpl<T>::kSlabSide);
  // pipelined exchange: the y/x stages of chunk k start when it has arrived;
  // within a chunk, plane ranges of at most interPlanes_ reuse the intermediate
  const bool pipe = pipelined();
  const int K = pipe ? exchChunks_ : 1;
  for (int k = 0; k < K; ++k) {
    if (pipe) chunkEv_[k]->wait_on(stream_);
    const int zb = pipe ? planeBounds_[k] : 0;
    const int ze = pipe ? planeBounds_[k + 1] : plan_->local_planes();
    for (int z0 = zb; z0 < ze; z0 += interPlanes_) {
      auto ya = yargs();
      auto xa = xargs();
      ya.zBegin = xa.zBegin = z0;
      ya.L = xa.L = std::min(ze, z0 + interPlanes_);
      if (pipe) {
        ya.colBase = colBaseChunk_[k] ? colBaseChunk_[k]->data<long long>() : nullptr;
        set_col_desc(ya, colDescChunk_[k]);
      }
      ya.plainSticks = plainHandoff_;
      cx<T>* in = inter_for(inter, z0);
      y_backward_launch(ya, slab, in);
      x_backward_launch(xa, in, space);
    }
  }
  if (outputLocation == SPFFT_PU_HOST) {
    gpu_check(hipMemcpyAsync(grid_->host_slot(GridImpl<T>::kSpace), space, space_bytes(),
                             hipMemcpyDeviceToHost, stream_),
              "hipMemcpyAsync");
  }
}

// ------------------------------------------------------------------- forward
template <typename T>
void GpuExecutor<T>::forward_xy(SpfftProcessingUnitType inputLocation) {
  SPFFT_TIMED_SCOPE("gpu_forward_xy");
  if (inputLocation != SPFFT_PU_HOST && inputLocation != SPFFT_PU_GPU)
    throw InvalidParameterError();
  DeviceGuard guard(deviceId_);
  order_after_default_stream();
  stage_mark("forward", nullptr);
  StageEnd stageEnd{this, "forward", "x+y"};
  void* space = grid_->device_slot(GridImpl<T>::kSpace);
  if (inputLocation == SPFFT_PU_HOST) {
    gpu_check(hipMemcpyAsync(space, grid_->host_slot(GridImpl<T>::kSpace), space_bytes(),
                             hipMemcpyHostToDevice, stream_),
              "hipMemcpyAsync");
  }
  poison(false);
  auto* inter = static_cast<cx<T>*>(grid_->device_slot(GridImpl<T>::kInter));
  void* slab = grid_->device_slot(GridImpl<T>::kSlabSide);
  // the y stage stores straight into the peers' stick sides
  if (peerWrites_) grid_->device_comm().prepare_write(GridImpl<T>::kStickSide, stream_);
  // pipelined exchange: chunk k's all-to-all starts when its y stage is done;
  // within a chunk, plane ranges of at most interPlanes_ reuse the intermediate
  const bool pipe = pipelined();
  const int K = pipe ? exchChunks_ : 1;
  for (int k = 0; k < K; ++k) {
    const int zb = pipe ? planeBounds_[k] : 0;
    const int ze = pipe ? planeBounds_[k + 1] : plan_->local_planes();
    for (int z0 = zb; z0 < ze; z0 += interPlanes_) {
      auto ya = yargs();
      auto xa = xargs();
      ya.zBegin = xa.zBegin = z0;
      ya.L = xa.L = std::min(ze, z0 + interPlanes_);
      if (pipe) {
        ya.colBase = colBaseChunk_[k] ? colBaseChunk_[k]->data<long long>() : nullptr;
        set_col_desc(ya, colDescChunk_[k]);
      } else if (peerWrites_) {
        ya.colBase = colBaseRemote_ ? colBaseRemote_->data<long long>() : nullptr;
        set_col_desc(ya, colDescRemote_);
      }
      cx<T>* out = inter_for(inter, z0);
      x_forward_launch(xa, space, out);
      y_forward_launch(ya, out, slab);
    }
    if (pipe) chunkEv_[k]->record(stream_);
  }
}

template <typename T>
void GpuExecutor<T>::forward_exchange(bool /*nonBlocking*/) {
  SPFFT_TIMED_SCOPE("gpu_forward_exchange");
  // pipelined: only the exchange's tail after the last y stage is left here
  StageEnd stageEnd{this, "forward", pipelined() ? "exchange-tail" : "exchange"};
  if (peerWrites_) {
    DeviceGuard guard(deviceId_);
    grid_->device_comm().complete_writes(stream_);
    return;
  }
  if (pipelined()) {
    pipelined_exchange(false);
    return;
  }
  exchange(false);
}

template <typename T>
void GpuExecutor<T>::forward_z(T* output, SpfftScalingType scaling) {
  SPFFT_TIMED_SCOPE("gpu_forward_z");
  DeviceGuard guard(deviceId_);
  StageEnd stageEnd{this, "forward", "z"};
  const IndexPlan& p = *plan_;
  const T factor =
      scaling == SPFFT_FULL_SCALING
          ? static_cast<T>(1.0 / (static_cast<double>(p.dimX) * p.dimY * p.dimZ))
          : T(1);
  cx<T>* values = reinterpret_cast<cx<T>*>(output);
  const bool hostOut = p.numLocalElements > 0 && !capturing_ && !is_device_pointer(output);
  if (p.numLocalElements > 0 && !output) throw InvalidParameterError();
  if (hostOut) values = staging(p.numLocalElements);
  const void* stick = grid_->device_slot(GridImpl<T>::kStickSide);
  auto a = zargs();
  if (peerWrites_) {
    grid_->device_comm().note_read(GridImpl<T>::kStickSide);
    a.single = 1;  // the single-rank stick layout (build_peer_tables)
    a.stickStride = peerStickStride_;
  }
  // pipelined plans: z(i) starts once stick block i has arrived
  const int I = pipelined() ? stickBlocks_ : 1;
  for (int i = 0; i < I; ++i) {
    if (pipelined()) {
      blockEv_[i]->wait_on(stream_);
      a.stickBegin = stickBounds_[i];
      a.numSticks = stickBounds_[i + 1];
    }
    if (longZ_ && floatExchange_)
      dev::launch_long_z_forward<T, cx<float>>(lpZ_, a, static_cast<const cx<float>*>(stick), values,
                                               factor, long_bufs(), stream_);
    else if (longZ_)
      dev::launch_long_z_forward<T, cx<T>>(lpZ_, a, static_cast<const cx<T>*>(stick), values, factor,
                                           long_bufs(), stream_);
    else if (floatExchange_)
      dev::launch_z_forward<T, cx<float>>(a, static_cast<const cx<float>*>(stick), values, factor,
                                          twZ_->data<cx<T>>(), stream_);
    else
      dev::launch_z_forward<T, cx<T>>(a, static_cast<const cx<T>*>(stick), values, factor,
                                      twZ_->data<cx<T>>(), stream_);
  }
  if (hostOut) {
    gpu_check(hipMemcpyAsync(output, values, sizeof(cx<T>) * p.numLocalElements,
                             hipMemcpyDeviceToHost, stream_),
              "hipMemcpyAsync");
  }
}

// ------------------------------------------------------- batched multi-transform
namespace {
struct Fnv {
  std::uint64_t h = 1469598103934665603ull;
  void bytes(const void* p, std::size_t n) {
    const unsigned char* c = static_cast<const unsigned char*>(p);
    for (std::size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  }
  template <typename U>
  void value(const U& v) { bytes(&v, sizeof(U)); }
  template <typename U>
  void vec(const std::vector<U>& v) {
    value(v.size());
    if (!v.empty()) bytes(v.data(), v.size() * sizeof(U));
  }
};
}  // namespace

// Everything the stage kernels read besides the data buffers: two transforms
// with equal keys can share one launch (and the first one's device tables).
template <typename T>
void GpuExecutor<T>::compute_batch_key() {
  const IndexPlan& p = *plan_;
  Fnv f;
  for (int v : {static_cast<int>(p.type), p.dimX, p.dimY, p.dimZ, p.numLocalElements, p.zeroStick,
                p.colOfX0, deviceId_, static_cast<int>(sizeof(T))})
    f.value(v);
  f.value(interStride_);
  f.vec(layout_.stickStride);
  f.vec(layout_.colEntryBase);
  f.value(layout_.slabStride);
  f.value(twXh_ != nullptr);
  f.vec(p.runs);
  f.vec(p.stickRunOffsets);
  f.vec(p.colX);
  f.vec(p.colOffsets);
  f.vec(p.colY);
  batchKey_ = f.h | 1;  // never 0
}

template <typename T>
bool GpuExecutor<T>::batchable() const {
  return batchEnabled_ && plan_->size == 1 && !peerWrites_ && !pipelined() && !capturing_ &&
         !poison_ && interPlanes_ >= plan_->local_planes() && !longX_ && !longY_ && !longZ_;
}

// A member needs no stream join when it runs on the leader's stream, or when
// both use their private streams synchronously: those are idle when a call
// starts (the previous call ended with a stream synchronize) and are
// synchronized again by multi_transform (the leader's covers the batch).
// Event joins cost ~3.4 us of host time per hipStreamWaitEvent on ROCm 7.2,
// more than the launches a batch saves on small grids
// (profiles/r2_s3/batch_ab.txt).
template <typename T>
bool GpuExecutor<T>::batch_join_free(const GpuExecutor& leader) const {
  if (stream_ == leader.stream_) return true;
  return ownStreamActive_ && synchronous_ && leader.ownStreamActive_ && leader.synchronous_;
}

template <typename T>
bool GpuExecutor<T>::batch_large() const {
  const IndexPlan& p = *plan_;
  return static_cast<long long>(p.dimX) * p.dimY * p.local_planes() >= batchLarge_;
}

// members on other streams: ordered after the default stream (private mode) and
// after their own streams' earlier work, then the leader's stream runs the batch
template <typename T>
void GpuExecutor<T>::batch_join(const std::vector<GpuExecutor*>& ex) {
  GpuExecutor* l = ex[0];
  l->order_after_default_stream();
  for (std::size_t i = 1; i < ex.size(); ++i) {
    GpuExecutor* e = ex[i];
    if (!e->batch_needs_join(*l)) continue;
    e->order_after_default_stream();
    if (!e->joinEvent_) e->joinEvent_.reset(new GpuEvent());
    e->joinEvent_->record(e->stream_);
    e->joinEvent_->wait_on(l->stream_);
  }
}

// joined members' streams wait for the batch, so later work on them sees it
template <typename T>
void GpuExecutor<T>::batch_release(const std::vector<GpuExecutor*>& ex) {
  GpuExecutor* l = ex[0];
  bool recorded = false;
  for (std::size_t i = 1; i < ex.size(); ++i) {
    GpuExecutor* e = ex[i];
    if (!e->batch_needs_join(*l)) continue;
    if (!recorded) {
      if (!l->doneEvent_) l->doneEvent_.reset(new GpuEvent());
      l->doneEvent_->record(l->stream_);
      recorded = true;
    }
    l->doneEvent_->wait_on(e->stream_);
  }
}

template <typename T>
void GpuExecutor<T>::backward_batch(const std::vector<GpuExecutor*>& ex,
                                    const std::vector<const T*>& inputs) {
  SPFFT_TIMED_SCOPE("gpu_backward_batch");
  const int n = static_cast<int>(ex.size());
  if (n < 1 || n > dev::kMaxBatch || inputs.size() != ex.size()) throw InternalError();
  GpuExecutor* l = ex[0];
  DeviceGuard guard(l->deviceId_);
  for (GpuExecutor* e : ex)
    if (!e->batchable() || e->batchKey_ != l->batchKey_) throw InternalError();
  batch_join(ex);
  const IndexPlan& p = *l->plan_;
  dev::BatchPtrs zb{}, yb{}, xb{};
  zb.count = yb.count = xb.count = n;
  for (int i = 0; i < n; ++i) {
    GpuExecutor* e = ex[i];
    if (p.numLocalElements > 0 && (!inputs[i] || !is_device_pointer(inputs[i])))
      throw InvalidParameterError();
    zb.in[i] = inputs[i];
    zb.out[i] = e->grid_->device_slot(GridImpl<T>::kStickSide);
    yb.in[i] = e->grid_->device_slot(GridImpl<T>::kSlabSide);
    yb.out[i] = e->grid_->device_slot(GridImpl<T>::kInter);
    xb.in[i] = yb.out[i];
    xb.out[i] = e->grid_->device_slot(GridImpl<T>::kSpace);
  }
  auto za = l->zargs();
  auto ya = l->yargs();
  auto xa = l->xargs();
  za.batch = zb;
  ya.batch = yb;
  xa.batch = xb;
  hipStream_t s = l->stream_;
  dev::launch_z_backward<T, cx<T>>(za, static_cast<const cx<T>*>(zb.in[0]),
                                   static_cast<cx<T>*>(zb.out[0]), l->twZ_->data<cx<T>>(), s);
  dev::launch_y_backward<T, cx<T>>(ya, static_cast<const cx<T>*>(yb.in[0]),
                                   static_cast<cx<T>*>(yb.out[0]), l->twY_->data<cx<T>>(), s);
  dev::launch_x_backward<T>(xa, p.type == SPFFT_TRANS_R2C, static_cast<const cx<T>*>(xb.in[0]),
                            xb.out[0], l->twX_->data<cx<T>>(),
                            l->twXh_ ? l->twXh_->data<cx<T>>() : nullptr, s);
  batch_release(ex);
}

template <typename T>
void GpuExecutor<T>::forward_batch(const std::vector<GpuExecutor*>& ex, const std::vector<T*>& outputs,
                                   SpfftScalingType scaling) {
  SPFFT_TIMED_SCOPE("gpu_forward_batch");
  const int n = static_cast<int>(ex.size());
  if (n < 1 || n > dev::kMaxBatch || outputs.size() != ex.size()) throw InternalError();
  GpuExecutor* l = ex[0];
  DeviceGuard guard(l->deviceId_);
  for (GpuExecutor* e : ex)
    if (!e->batchable() || e->batchKey_ != l->batchKey_) throw InternalError();
  batch_join(ex);
  const IndexPlan& p = *l->plan_;
  const T factor = scaling == SPFFT_FULL_SCALING
                       ? static_cast<T>(1.0 / (static_cast<double>(p.dimX) * p.dimY * p.dimZ))
                       : T(1);
  dev::BatchPtrs zb{}, yb{}, xb{};
  zb.count = yb.count = xb.count = n;
  for (int i = 0; i < n; ++i) {
    GpuExecutor* e = ex[i];
    if (p.numLocalElements > 0 && (!outputs[i] || !is_device_pointer(outputs[i])))
      throw InvalidParameterError();
    xb.in[i] = e->grid_->device_slot(GridImpl<T>::kSpace);
    xb.out[i] = e->grid_->device_slot(GridImpl<T>::kInter);
    yb.in[i] = xb.out[i];
    yb.out[i] = e->grid_->device_slot(GridImpl<T>::kSlabSide);
    zb.in[i] = e->grid_->device_slot(GridImpl<T>::kStickSide);
    zb.out[i] = outputs[i];
  }
  auto za = l->zargs();
  auto ya = l->yargs();
  auto xa = l->xargs();
  za.batch = zb;
  ya.batch = yb;
  xa.batch = xb;
  hipStream_t s = l->stream_;
  dev::launch_x_forward<T>(xa, p.type == SPFFT_TRANS_R2C, xb.in[0], static_cast<cx<T>*>(xb.out[0]),
                           l->twX_->data<cx<T>>(), l->twXh_ ? l->twXh_->data<cx<T>>() : nullptr, s);
  dev::launch_y_forward<T, cx<T>>(ya, static_cast<const cx<T>*>(yb.in[0]),
                                  static_cast<cx<T>*>(yb.out[0]), l->twY_->data<cx<T>>(), s);
  dev::launch_z_forward<T, cx<T>>(za, static_cast<const cx<T>*>(zb.in[0]),
                                  static_cast<cx<T>*>(zb.out[0]), factor, l->twZ_->data<cx<T>>(), s);
  batch_release(ex);
}

template class GpuExecutor<double>;
template class GpuExecutor<float>;

}  // namespace spfft
