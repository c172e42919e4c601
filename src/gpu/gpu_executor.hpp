// GPU execution engine (reference: src/execution/execution_gpu.{hpp,cpp}).
//
// Per direction three fused kernels (z, y, x stage) plus, for distributed
// grids, one RCCL all-to-all(v) — all enqueued on one HIP stream without host
// synchronisation; the call blocks only at the end (synchronous mode, the
// SpFFT contract) or never (asynchronous mode with a user stream).
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

#include "api/grid_impl.hpp"
#include "gpu/device_comm.hpp"
#include "gpu/gpu_runtime.hpp"
#include "kernels/long_fft.hpp"
#include "kernels/stage_args.hpp"
#include "plan/index_plan.hpp"

namespace spfft {

template <typename T>
class GpuExecutor {
public:
  GpuExecutor(std::shared_ptr<GridImpl<T>> grid, std::shared_ptr<const IndexPlan> plan);
  ~GpuExecutor();

  void backward_z(const T* input);
  void backward_exchange(bool nonBlocking);
  void backward_xy(SpfftProcessingUnitType outputLocation);
  void forward_xy(SpfftProcessingUnitType inputLocation);
  void forward_exchange(bool nonBlocking);
  void forward_z(T* output, SpfftScalingType scaling);

  // Whole-direction hipGraph replay (single-rank transforms with device-resident
  // input and output): the direction's launches are captured once per
  // (pointers, scaling, stream) and replayed with one hipGraphLaunch. Returns
  // false (nothing enqueued) when the call is not eligible; the caller then runs
  // the step-wise path. Opt-in with SPFFT_GRAPH=1.
  bool backward_graph(const T* input, SpfftProcessingUnitType outputLocation);
  bool forward_graph(SpfftProcessingUnitType inputLocation, T* output, SpfftScalingType scaling);

  // Batched multi-transform: single-rank transforms on one device whose plans
  // are identical (same dimensions, type, index set and layout knobs: equal
  // batch_key()) run each stage of a direction as ONE launch for up to
  // dev::kMaxBatch transforms (blockIdx.z = transform). Small grids are
  // latency bound per launch; a batch fills the GPU (SPFFT_BATCH=0 disables).
  // The batch runs on ex[0]'s stream. Members on other streams are joined by
  // events, which costs more host time than the saved launches on small grids:
  // there only join-free members are batched (batch_join_free). Large grids
  // (batch_large: GPU bound, the joins hide behind the kernels) are batched in
  // sub-batches of batch_split() on their leaders' streams, so the stages of
  // different sub-batches overlap. Inputs/outputs must be device pointers.
  bool batchable() const;
  bool batch_join_free(const GpuExecutor& leader) const;
  bool batch_large() const;
  int batch_split() const { return batchSplit_; }
  std::uint64_t batch_key() const { return batchKey_; }
  static void backward_batch(const std::vector<GpuExecutor*>& ex, const std::vector<const T*>& inputs);
  static void forward_batch(const std::vector<GpuExecutor*>& ex, const std::vector<T*>& outputs,
                            SpfftScalingType scaling);

  void synchronize();
  bool synchronous() const { return synchronous_; }
  // Execute on `stream` (nullptr = the legacy default stream); work is then
  // ordered by the stream itself. reset_stream() returns to the private stream,
  // which is ordered after the default stream with an event per call.
  void set_stream(hipStream_t stream, bool synchronous);
  void reset_stream();
  hipStream_t stream() const { return stream_; }
  // Creates the private stream now if the transform runs on it (it is
  // otherwise created by the first call).
  void ensure_stream() { use_private_stream(); }
  T* space_domain(SpfftProcessingUnitType location);

private:
  template <typename U>
  U* upload(std::unique_ptr<DeviceBuffer>& buf, const std::vector<U>& v);
  void order_after_default_stream();
  void use_private_stream();  // creates the private stream on first use
  void z_backward_launch(const dev::ZArgs& a, const cx<T>* values, void* stick);
  void exchange(bool backward);
  void build_peer_tables();
  bool build_chunk_plan(int chunks, int blocks);
  bool chunk_plan_fits(int chunks) const;
  void pipelined_exchange(bool backward);
  void wait_stream();
  void wait_stream_watched();
  void log_plan() const;
  void poison(bool backward);
  dev::ZArgs zargs() const;
  dev::YArgs yargs() const;
  dev::XArgs xargs() const;
  cx<T>* staging(std::size_t elems);
  struct GraphEntry {
    int dir;  // 0 backward, 1 forward
    const void* in;
    const void* out;
    int scaling;
    hipStream_t stream;
    hipGraphExec_t exec;
  };
  bool graph_eligible() const;
  template <class Enqueue>
  bool replay(const GraphEntry& key, Enqueue enqueue);
  std::size_t space_bytes() const;

  std::shared_ptr<GridImpl<T>> grid_;
  std::shared_ptr<const IndexPlan> plan_;
  ExchangeLayout layout_;
  bool floatExchange_ = false;
  long long interStride_ = 0;  // row stride of [z][column][y]
  int interPlanes_ = 1;        // planes per y/x launch pair (fits the grid's intermediate)
  // axes beyond one workgroup's LDS: glue + global four-step / Bluestein FFT
  bool longX_ = false, longY_ = false, longZ_ = false;
  dev::LongPlan lpX_, lpY_, lpZ_;
  std::unique_ptr<DeviceBuffer> longWork_[4];
  void setup_long_axes();
  dev::LongBufs<T> long_bufs() const;
  void y_backward_launch(const dev::YArgs& ya, const void* slab, cx<T>* inter);
  void y_forward_launch(const dev::YArgs& ya, cx<T>* inter, void* slab);
  void x_backward_launch(const dev::XArgs& xa, const cx<T>* inter, void* space);
  void x_forward_launch(const dev::XArgs& xa, const void* space, cx<T>* inter);
  cx<T>* inter_for(cx<T>* inter, int z0) const;
  bool poison_ = false;        // SPFFT_POISON=1: NaN-fill work buffers before each direction
  int deviceId_ = 0;

  std::unique_ptr<GpuStream> ownStream_;
  hipStream_t stream_ = nullptr;
  bool ownStreamActive_ = true;
  bool synchronous_ = true;
  std::unique_ptr<GpuEvent> event_;
  std::uint64_t batchKey_ = 0;
  bool batchEnabled_ = true;
  long long batchLarge_ = 0;  // slab elements from which joins are allowed
  int batchSplit_ = 2;        // sub-batch size of large grids
  std::unique_ptr<GpuEvent> joinEvent_, doneEvent_;
  static void batch_join(const std::vector<GpuExecutor*>& ex);
  static void batch_release(const std::vector<GpuExecutor*>& ex);
  bool batch_needs_join(const GpuExecutor& leader) const {
    return stream_ != leader.stream_ && !batch_join_free(leader);
  }
  void compute_batch_key();
  bool capturing_ = false;      // order/poison steps are skipped inside a capture
  bool graphsEnabled_ = false;  // SPFFT_GRAPH=1; off again after a failed capture
  bool warm_[2] = {false, false};  // first call of a direction runs eagerly
  std::vector<GraphEntry> graphs_;

  // device tables
  std::unique_ptr<DeviceBuffer> runs_, runOffsets_, descs_;
  // exchange segments of the z stage: segment v holds planes [segZOff, +n) of
  // its sticks at segDispl[v] + s * segStride[v]; the device table (ZArgs::zTab)
  // has one (base, stride) entry per plane
  std::vector<int> zSeg_, segZOff_;
  std::vector<long long> segStride_;
  std::unique_ptr<DeviceBuffer> zTab_, zTabRemote_;
  void upload_ztab(std::unique_ptr<DeviceBuffer>& dst, const std::vector<long long>& segDispl);
  std::unique_ptr<DeviceBuffer> colOffsets_, colY_, colBase_, colX_, xToCol_;
  // per-column run descriptors of the y stage (YArgs::colDesc), one per colBase
  // table in use; null when some column needs more than kColRuns runs.
  // SPFFT_COL_DESC=0 disables them.
  struct ColDescTable {
    std::unique_ptr<DeviceBuffer> buf;
    long long stride = 0;
    const dev::ColDesc* ptr() const { return buf ? buf->data<dev::ColDesc>() : nullptr; }
  };
  bool colDescs_ = true;
  ColDescTable colDesc_, colDescRemote_;
  std::vector<ColDescTable> colDescChunk_;
  void build_col_desc(ColDescTable& t, const std::vector<long long>& colBase, long long stride);
  void set_col_desc(dev::YArgs& a, const ColDescTable& t) const {
    a.colDesc = t.ptr();
    a.colStride = t.stride;
  }
  // peer-write exchange (DeviceComm::peer_writes): the z stage (backward) and y
  // stage (forward) store straight into the receivers' buffers; these tables
  // hold those destinations as element offsets from the local buffer.
  bool peerWrites_ = false;
  // RCCL / loopback data planes: this rank's own exchange block is written in
  // place on the slab side instead of being copied (SPFFT_LOCAL_DIRECT=0 copies)
  bool localDirect_ = false;
  long long slab_offset() const;
  std::unique_ptr<DeviceBuffer> colBaseRemote_;
  long long peerOffsetRange_[2] = {0, 0};  // min / max remote base (SPFFT_LOG)

  // Pipelined exchange (RCCL / loopback data planes): a 2D grid of I stick
  // blocks x K plane chunks. Both exchange buffers are laid out chunk-major
  // (chunk k is one contiguous block per peer), and inside a block the rows are
  // sticks, so message (i, k) to or from a peer is one contiguous byte range on
  // both sides. Backward: the z stage runs per stick block; the messages of
  // block i leave as soon as z(i) is done (overlapping z(i+1)); the last
  // block's messages go out chunk by chunk and the y/x stages of chunk k start
  // once chunk k has arrived. Forward is the mirror image: x/y per chunk, chunk
  // k leaves when its y stage is done, the last chunk goes out block by block
  // and z(i) starts once block i has arrived. Every exchange runs on the data
  // plane's channel stream (RCCL: one per process, in host call order), handed
  // off by one event per step: a rank with T transforms uses T + 1 streams.
  struct ExchangeStep {
    std::vector<Transfer> xs;  // transfer list of the step (backward direction)
    int readyKind, readyIdx;   // event the step waits for: 0 none, 1 zEv_[i], 2 chunkEv_[k]
    int doneKind, doneIdx;     // event recorded after it: 0 none, 2 chunkEv_[k], 3 blockEv_[i]
    int id = -1;               // registered with the data plane (DeviceComm::register_exchange)
  };
  // registers every exchange of the plan with the data plane (collective)
  void register_exchanges();
  int bwdId_ = -1, fwdId_ = -1;  // registered unpipelined exchanges
  int plainHandoff_ = 0;         // backward stick hand-off through the Infinity Cache
  long long peerStickStride_ = 0;  // peer writes: stick row stride of the stick side
  int exchChunks_ = 1;   // K
  int stickBlocks_ = 1;  // I
  bool pipelined() const { return exchChunks_ > 1 || stickBlocks_ > 1; }

public:
  // The exchange plan (plane chunks K x stick blocks I; peer writes), for
  // bench.py's modelled times and SPFFT_LOG.
  int exchange_chunks() const { return exchChunks_; }
  int exchange_stick_blocks() const { return stickBlocks_; }
  bool exchange_peer_writes() const { return peerWrites_; }

private:
  double chunkModel_ = 0;  // per-peer bytes of one exchange (chunk model input)
  std::vector<int> planeBounds_;  // K+1 local plane bounds of the chunks
  std::vector<int> stickBounds_;  // I+1 local stick bounds of the z launches
  std::vector<ExchangeStep> bwdSteps_, fwdSteps_;
  std::vector<std::unique_ptr<DeviceBuffer>> colBaseChunk_;  // y-stage entry bases per chunk
  std::vector<std::unique_ptr<GpuEvent>> zEv_, chunkEv_, blockEv_;
  hipEvent_t step_event(int kind, int idx) const;
  void run_steps(const std::vector<ExchangeStep>& steps, bool backward);
  // GPU-side stage timing (SPFFT_TIMING=1): timing events recorded on the
  // execution stream at the stage boundaries of each direction; the intervals
  // go into the timing tree as gpu/<direction>/<stage> once they completed.
  struct StageMark {
    std::unique_ptr<GpuEvent> ev;
    const char* stage;  // stage that ends at this mark (nullptr: direction start)
  };
  struct StageTrace {
    const char* dir;
    std::vector<StageMark> marks;
  };
  std::vector<StageTrace> traces_;
  struct ExchangeSpan {
    const char* dir;
    std::unique_ptr<GpuEvent> begin, end;
  };
  std::vector<ExchangeSpan> spans_;  // pipelined exchanges (gpu/<dir>/exchange-span)
  std::vector<std::unique_ptr<GpuEvent>> spareEvents_;
  std::unique_ptr<GpuEvent> timing_event();
  void stage_mark(const char* dir, const char* stage);
  // records the end mark of a stage when the stage function returns
  struct StageEnd {
    GpuExecutor* e;
    const char* dir;
    const char* stage;
    ~StageEnd() {
      if (!stage) return;  // nothing ends here
      try {
        e->stage_mark(dir, stage);
      } catch (...) {
      }
    }
  };
  void harvest_stage_times(bool wait);

  std::unique_ptr<DeviceBuffer> twX_, twXh_, twY_, twZ_;
  std::unique_ptr<DeviceBuffer> staging_;
  std::vector<std::int64_t> bwdSendCounts_, bwdSendDispls_, bwdRecvCounts_, bwdRecvDispls_;
};

}  // namespace spfft
