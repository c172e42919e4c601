// IndexPlan: frequency-index validation, z-stick discovery, distribution
// metadata and the tables the host/GPU stage kernels consume.
//
// Semantics follow SpFFT (reference: src/compression/indices.hpp:49-186,
// src/parameters/parameters.cpp:43-180): sticks are ordered by the key
// x*dimY + y of their storage indices, centred indices are detected if ANY
// index is negative, R2C restricts x to [0, dimX/2], duplicate sticks across
// ranks are an error, planes are assigned to ranks in rank order.
//
// Representation is new: instead of one stick-slot index per value, values are
// grouped into runs (contiguous in value order AND in z) so the fused GPU
// z-stage can gather/scatter whole runs with coalesced accesses.
#pragma once

#include <cstdint>
#include <vector>

#include "core/common.hpp"
#include "spfft/communicator.hpp"
#include "spfft/types.h"

namespace spfft {

struct StickRun {
  std::int32_t valueStart;  // first value index of the run
  std::int32_t zStart;      // storage z of the first value
  std::int32_t length;      // number of values (z contiguous, no wrap)
  std::int32_t stick;       // local stick index
};

// Per-stick descriptor for the common case where a stick's values are
// contiguous in value order and form at most two z-runs (e.g. a centred
// sphere: z = 0..h then n-h..n-1). Lets the z-stage map (stick, j) -> (value,
// z) with two compares instead of a run search.
struct StickDesc {
  std::int32_t valueStart;  // first value of the stick
  std::int32_t count;       // number of values
  std::int32_t z0;          // storage z of value j < len0 is z0 + j
  std::int32_t len0;
  std::int32_t z1;          // storage z of value j >= len0 is z1 + (j - len0)
  std::int32_t pad[3];
};

class IndexPlan {
public:
  // comm == nullptr (or size 1 and localZLength == dimZ) -> local plan.
  IndexPlan(Communicator* comm, SpfftTransformType type, int dimX, int dimY, int dimZ,
            int localZLength, int numLocalElements, SpfftIndexFormatType format,
            const int* indices);

  SpfftTransformType type;
  int dimX, dimY, dimZ, dimXFreq;
  int rank = 0, size = 1;

  std::vector<int> sticksPerRank, planesPerRank, planeOffsets;
  std::vector<std::vector<int>> stickKeysPerRank;  // sorted keys x*dimY+y (storage indices)
  int maxSticks = 0, maxPlanes = 0;                 // over all ranks
  int numLocalElements = 0;
  long long numGlobalElements = 0;
  long long totalSticks = 0;

  // local sticks
  int local_sticks() const { return sticksPerRank[rank]; }
  int local_planes() const { return planesPerRank[rank]; }
  int local_plane_offset() const { return planeOffsets[rank]; }
  std::vector<StickRun> runs;         // grouped by stick (stable in value order)
  std::vector<int> stickRunOffsets;   // local_sticks()+1
  int zeroStick = -1;                 // local index of the (0,0) stick, -1 if not local
  std::vector<StickDesc> stickDescs;  // filled when every local stick is "simple"
  bool simpleSticks = false;

  // x-columns over ALL ranks' sticks (the y-stage works on these)
  std::vector<int> colX;        // storage x of column c, ascending
  std::vector<int> colOffsets;  // ncols+1, entries sorted by y
  std::vector<int> colY;        // per entry: storage y
  std::vector<int> colRank;     // per entry: owning rank
  std::vector<int> colLocal;    // per entry: stick index on the owning rank
  std::vector<int> xToCol;      // dimXFreq entries, -1 where no column
  int colOfX0 = -1;             // column with x == 0 (R2C plane symmetry), -1 if none
  int num_columns() const { return static_cast<int>(colX.size()); }
};

// Layout of the two exchange-side buffers (elements of complex type).
//  stick side: block r holds (local sticks) x (planes of rank r); stick s,
//              plane z of rank r at stickDispl[r] + s*stickStride[r] + (z - planeOffsets[r]).
//  slab side:  block r holds (sticks of rank r) x (local planes); entry base
//              colEntryBase[k] + zLocal.
// With one rank both sides are the plain stick array [S][dimZ].
struct ExchangeLayout {
  bool buffered = false;
  std::vector<i64> stickDispl, stickStride, stickCount;
  std::vector<i64> slabDispl, slabCount;
  i64 slabStride = 0;
  i64 stickTotal = 0, slabTotal = 0;
  std::vector<i64> colEntryBase;
};

// stickPad: extra elements between sticks of the single-rank layout (breaks the
// power-of-two stride of [S][dimZ]; HBM channel spreading).
ExchangeLayout make_exchange_layout(const IndexPlan& plan, bool buffered, int stickPad = 0);

}  // namespace spfft
