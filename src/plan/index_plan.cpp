#include "plan/index_plan.hpp"

#include <algorithm>
#include <cstring>
#include <numeric>
#include <tuple>
#include <unordered_map>

#include "spfft/exceptions.hpp"

namespace spfft {
namespace {

inline int to_storage(int dim, int idx) { return idx < 0 ? idx + dim : idx; }

// Status codes exchanged before any data-dependent collective, so that an
// error on one rank does not leave the others blocked (the reference throws
// before its collectives, src/compression/indices.hpp:120-149).
enum : std::int64_t { kOk = 0, kInvalidParam = 1, kInvalidIndices = 2, kInternal = 3 };

[[noreturn]] void throw_status(std::int64_t st) {
  switch (st) {
    case kInvalidParam: throw InvalidParameterError();
    case kInvalidIndices: throw InvalidIndicesError();
    case kInternal: throw InternalError();
    default: throw MPIParameterMismatchError();
  }
}

struct LocalConversion {
  std::int64_t status = kOk;
  std::vector<int> keys;  // sorted unique stick keys
  std::vector<StickRun> runs;
  std::vector<int> runOffsets;
};

LocalConversion convert_triplets(bool hermitian, int dimX, int dimY, int dimZ, int n,
                                 SpfftIndexFormatType format, const int* idx) {
  LocalConversion out;
  if (format != SPFFT_INDEX_TRIPLETS) {
    out.status = kInternal;
    return out;
  }
  if (n < 0 || static_cast<long long>(n) >
                   static_cast<long long>(dimX) * static_cast<long long>(dimY) * dimZ) {
    out.status = kInvalidParam;
    return out;
  }
  bool centered = false;
  for (long long i = 0; i < 3LL * n; ++i) {
    if (idx[i] < 0) {
      centered = true;
      break;
    }
  }
  const int maxX = (hermitian || centered ? dimX / 2 + 1 : dimX) - 1;
  const int maxY = (centered ? dimY / 2 + 1 : dimY) - 1;
  const int maxZ = (centered ? dimZ / 2 + 1 : dimZ) - 1;
  const int minX = hermitian ? 0 : maxX - dimX + 1;
  const int minY = maxY - dimY + 1;
  const int minZ = maxZ - dimZ + 1;
  for (int i = 0; i < n; ++i) {
    const int x = idx[3 * i], y = idx[3 * i + 1], z = idx[3 * i + 2];
    if (x < minX || x > maxX || y < minY || y > maxY || z < minZ || z > maxZ) {
      out.status = kInvalidIndices;
      return out;
    }
  }

  // stick key -> local slot
  const long long planeSize = static_cast<long long>(dimX) * dimY;
  std::vector<int> slotOfValue(static_cast<std::size_t>(n));
  if (planeSize <= (1LL << 26)) {
    std::vector<int> dense(static_cast<std::size_t>(planeSize), -1);
    for (int i = 0; i < n; ++i) {
      const int key = to_storage(dimX, idx[3 * i]) * dimY + to_storage(dimY, idx[3 * i + 1]);
      dense[key] = 0;
    }
    int count = 0;
    for (long long k = 0; k < planeSize; ++k) {
      if (dense[k] == 0) {
        dense[k] = count++;
        out.keys.push_back(static_cast<int>(k));
      }
    }
    for (int i = 0; i < n; ++i) {
      const int key = to_storage(dimX, idx[3 * i]) * dimY + to_storage(dimY, idx[3 * i + 1]);
      slotOfValue[i] = dense[key];
    }
  } else {
    std::vector<int> keyOfValue(static_cast<std::size_t>(n));
    for (int i = 0; i < n; ++i)
      keyOfValue[i] = to_storage(dimX, idx[3 * i]) * dimY + to_storage(dimY, idx[3 * i + 1]);
    out.keys = keyOfValue;
    std::sort(out.keys.begin(), out.keys.end());
    out.keys.erase(std::unique(out.keys.begin(), out.keys.end()), out.keys.end());
    for (int i = 0; i < n; ++i)
      slotOfValue[i] = static_cast<int>(
          std::lower_bound(out.keys.begin(), out.keys.end(), keyOfValue[i]) - out.keys.begin());
  }

  // runs in value order, then grouped by stick with a stable counting sort
  std::vector<StickRun> runs;
  for (int i = 0; i < n; ++i) {
    const int s = slotOfValue[i];
    const int z = to_storage(dimZ, idx[3 * i + 2]);
    if (!runs.empty()) {
      StickRun& r = runs.back();
      if (r.stick == s && r.zStart + r.length == z && r.valueStart + r.length == i) {
        ++r.length;
        continue;
      }
    }
    runs.push_back(StickRun{i, z, 1, s});
  }
  const int S = static_cast<int>(out.keys.size());
  out.runOffsets.assign(S + 1, 0);
  for (const auto& r : runs) ++out.runOffsets[r.stick + 1];
  for (int s = 0; s < S; ++s) out.runOffsets[s + 1] += out.runOffsets[s];
  out.runs.resize(runs.size());
  std::vector<int> fill(out.runOffsets.begin(), out.runOffsets.end() - 1);
  for (const auto& r : runs) out.runs[fill[r.stick]++] = r;
  return out;
}

}  // namespace

IndexPlan::IndexPlan(Communicator* comm, SpfftTransformType t, int dX, int dY, int dZ,
                     int localZLength, int numLocal, SpfftIndexFormatType format,
                     const int* indices)
    : type(t), dimX(dX), dimY(dY), dimZ(dZ), dimXFreq(t == SPFFT_TRANS_R2C ? dX / 2 + 1 : dX) {
  if (t != SPFFT_TRANS_C2C && t != SPFFT_TRANS_R2C) throw InvalidParameterError();
  if (dX < 1 || dY < 1 || dZ < 1 || localZLength < 0 || numLocal < 0)
    throw InvalidParameterError();
  if (numLocal > 0 && !indices) throw InvalidParameterError();

  LocalConversion conv =
      convert_triplets(t == SPFFT_TRANS_R2C, dX, dY, dZ, numLocal, format, indices);

  const bool distributed = comm && comm->size() > 1;
  if (!distributed) {
    if (conv.status != kOk) throw_status(conv.status);
    rank = 0;
    size = 1;
    sticksPerRank = {static_cast<int>(conv.keys.size())};
    planesPerRank = {localZLength};
    planeOffsets = {0};
    numGlobalElements = numLocal;
    stickKeysPerRank.push_back(conv.keys);
    if (localZLength != dZ) throw InvalidParameterError();
  } else {
    rank = comm->rank();
    size = comm->size();
    // 1) status + per-rank parameters
    struct Params {
      std::int64_t status, dimX, dimY, dimZ, planes, sticks, elements;
    };
    Params mine{conv.status, dX, dY, dZ, localZLength,
                static_cast<std::int64_t>(conv.keys.size()), numLocal};
    std::vector<Params> all(size);
    comm->allgather(&mine, all.data(), sizeof(Params));
    for (const auto& p : all) {
      if (p.status != kOk) {
        if (conv.status != kOk) throw_status(conv.status);
        throw MPIParameterMismatchError();
      }
    }
    long long sumPlanes = 0, sumSticks = 0;
    for (const auto& p : all) {
      if (p.dimX != dX || p.dimY != dY || p.dimZ != dZ) throw MPIParameterMismatchError();
      sumPlanes += p.planes;
      sumSticks += p.sticks;
    }
    if (sumSticks > static_cast<long long>(dX) * dY) throw MPIParameterMismatchError();
    if (sumPlanes != dZ) throw MPIParameterMismatchError();
    int offset = 0;
    for (const auto& p : all) {
      sticksPerRank.push_back(static_cast<int>(p.sticks));
      planesPerRank.push_back(static_cast<int>(p.planes));
      planeOffsets.push_back(offset);
      offset += static_cast<int>(p.planes);
      numGlobalElements += p.elements;
    }
    // 2) stick keys of every rank (padded allgather)
    const int maxS = *std::max_element(sticksPerRank.begin(), sticksPerRank.end());
    std::vector<int> sendKeys(static_cast<std::size_t>(std::max(1, maxS)), -1);
    std::copy(conv.keys.begin(), conv.keys.end(), sendKeys.begin());
    std::vector<int> recvKeys(sendKeys.size() * size);
    comm->allgather(sendKeys.data(), recvKeys.data(), sendKeys.size() * sizeof(int));
    stickKeysPerRank.resize(size);
    for (int r = 0; r < size; ++r) {
      const int* b = recvKeys.data() + static_cast<std::size_t>(r) * sendKeys.size();
      stickKeysPerRank[r].assign(b, b + sticksPerRank[r]);
    }
    // duplicates across ranks
    std::vector<int> allKeys;
    for (const auto& k : stickKeysPerRank) allKeys.insert(allKeys.end(), k.begin(), k.end());
    std::sort(allKeys.begin(), allKeys.end());
    if (std::adjacent_find(allKeys.begin(), allKeys.end()) != allKeys.end())
      throw DuplicateIndicesError();
  }

  numLocalElements = numLocal;
  runs = std::move(conv.runs);
  stickRunOffsets = std::move(conv.runOffsets);
  {
    // stick descriptors (simple sticks: values contiguous, <= 2 z-runs)
    const int S = static_cast<int>(stickRunOffsets.size()) - 1;
    simpleSticks = true;
    stickDescs.assign(std::max(0, S), StickDesc{});
    for (int s = 0; s < S && simpleSticks; ++s) {
      const int q0 = stickRunOffsets[s], q1 = stickRunOffsets[s + 1];
      const int nr = q1 - q0;
      StickDesc d{};
      if (nr == 0 || nr > 2) {
        simpleSticks = nr == 0;
        stickDescs[s] = d;
        continue;
      }
      const StickRun& a = runs[q0];
      d.valueStart = a.valueStart;
      d.count = a.length;
      d.z0 = a.zStart;
      d.len0 = a.length;
      d.z1 = 0;
      if (nr == 2) {
        const StickRun& b = runs[q0 + 1];
        if (b.valueStart != a.valueStart + a.length) simpleSticks = false;
        d.count += b.length;
        d.z1 = b.zStart;
      }
      stickDescs[s] = d;
    }
    if (!simpleSticks) stickDescs.clear();
  }
  maxSticks = *std::max_element(sticksPerRank.begin(), sticksPerRank.end());
  maxPlanes = *std::max_element(planesPerRank.begin(), planesPerRank.end());
  for (int s : sticksPerRank) totalSticks += s;
  {
    const auto& mk = stickKeysPerRank[rank];
    auto it = std::lower_bound(mk.begin(), mk.end(), 0);
    zeroStick = (it != mk.end() && *it == 0) ? static_cast<int>(it - mk.begin()) : -1;
  }

  // columns
  struct Entry {
    int x, y, r, s;
  };
  std::vector<Entry> entries;
  entries.reserve(static_cast<std::size_t>(totalSticks));
  for (int r = 0; r < size; ++r) {
    const auto& keys = stickKeysPerRank[r];
    for (int s = 0; s < static_cast<int>(keys.size()); ++s)
      entries.push_back(Entry{keys[s] / dY, keys[s] % dY, r, s});
  }
  std::sort(entries.begin(), entries.end(),
            [](const Entry& a, const Entry& b) { return std::tie(a.x, a.y) < std::tie(b.x, b.y); });
  xToCol.assign(dimXFreq, -1);
  for (const auto& e : entries) {
    if (colX.empty() || colX.back() != e.x) {
      colX.push_back(e.x);
      colOffsets.push_back(static_cast<int>(colY.size()));
    }
    colY.push_back(e.y);
    colRank.push_back(e.r);
    colLocal.push_back(e.s);
  }
  colOffsets.push_back(static_cast<int>(colY.size()));
  for (int c = 0; c < num_columns(); ++c) {
    if (colX[c] < dimXFreq) xToCol[colX[c]] = c;
    if (colX[c] == 0) colOfX0 = c;
  }
}

ExchangeLayout make_exchange_layout(const IndexPlan& p, bool buffered, int stickPad) {
  ExchangeLayout l;
  const int P = p.size;
  const i64 S = p.local_sticks();
  const i64 L = p.local_planes();
  l.buffered = buffered && P > 1;
  l.stickDispl.resize(P);
  l.stickStride.resize(P);
  l.stickCount.resize(P);
  l.slabDispl.resize(P);
  l.slabCount.resize(P);
  if (P == 1) {
    l.stickDispl[0] = 0;
    l.stickStride[0] = p.dimZ + stickPad;
    l.stickCount[0] = S * (p.dimZ + stickPad);
    l.slabDispl[0] = 0;
    l.slabStride = p.dimZ + stickPad;
    l.slabCount[0] = S * (p.dimZ + stickPad);
  } else if (l.buffered) {
    const i64 block = static_cast<i64>(p.maxSticks) * p.maxPlanes;
    for (int r = 0; r < P; ++r) {
      l.stickDispl[r] = r * block;
      l.stickStride[r] = p.maxPlanes;
      l.stickCount[r] = block;
      l.slabDispl[r] = r * block;
      l.slabCount[r] = block;
    }
    l.slabStride = p.maxPlanes;
  } else {
    i64 so = 0, ro = 0;
    for (int r = 0; r < P; ++r) {
      l.stickDispl[r] = so;
      l.stickStride[r] = p.planesPerRank[r];
      l.stickCount[r] = S * p.planesPerRank[r];
      so += l.stickCount[r];
      l.slabDispl[r] = ro;
      l.slabCount[r] = static_cast<i64>(p.sticksPerRank[r]) * L;
      ro += l.slabCount[r];
    }
    l.slabStride = L;
  }
  l.stickTotal = std::accumulate(l.stickCount.begin(), l.stickCount.end(), i64(0));
  l.slabTotal = std::accumulate(l.slabCount.begin(), l.slabCount.end(), i64(0));
  l.colEntryBase.resize(p.colY.size());
  for (std::size_t k = 0; k < p.colY.size(); ++k)
    l.colEntryBase[k] = l.slabDispl[p.colRank[k]] + static_cast<i64>(p.colLocal[k]) * l.slabStride;
  return l;
}

}  // namespace spfft
