// Stage launchers (templates): one workgroup engine per line length, the
// kernel's LDS and grid, and the launch. Explicit instantiations live in one
// translation unit per stage and precision (z/y/x_stage*.hip), so the stage
// kernels compile in parallel.
// The packed-real R2C x stage runs forward on the row-mapped engine (the first
// FFT pass loads the real rows directly) rather than the line-fast one with the
// rows staged through LDS: 58.9 -> 56.8 us at 256^3 (profiles/r2_s1/shape_ab.txt).
#pragma once

#include "kernels/stage_kernels.hpp"

namespace spfft {
namespace dev {


template <typename T, typename BT>
void launch_z_backward(const ZArgs& a, const cx<T>* values, BT* out, const cx<T>* tw,
                       hipStream_t stream) {
  if (a.numSticks <= a.stickBegin) return;
  with_engine<T, +1>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    using E = decltype(eng);
    // (plain stick stores only where the executor asks for them: plainSticks)
    const bool plain = a.plainSticks != 0;
    auto k = !a.desc ? z_backward_kernel<E, T, BT>
             : plain ? z_backward_desc_kernel<E, T, BT, true> : z_backward_desc_kernel<E, T, BT, false>;
    std::size_t ldsTotal = 0;
    const ZArgs b = z_args_for_lds(a, lds, lines, &ldsTotal);
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.numSticks - a.stickBegin, lines), 1, batch_dim(a.batch)), dim3(threads),
                       ldsTotal, stream, eng, b, values, out, tw);
    gpu_check_launch("z_backward", stream);
  });
}

template <typename T, typename BT>
void launch_z_forward(const ZArgs& a, const BT* in, cx<T>* values, T scale, const cx<T>* tw,
                      hipStream_t stream) {
  if (a.numSticks <= a.stickBegin) return;
  with_engine<T, -1>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    using E = decltype(eng);
    auto k = !a.desc ? z_forward_kernel<E, T, BT>
             : a.ntValueStores ? z_forward_desc_kernel<E, T, BT, true> : z_forward_desc_kernel<E, T, BT, false>;
    std::size_t ldsTotal = 0;
    const ZArgs b = z_args_for_lds(a, lds, lines, &ldsTotal);
    prepare_kernel(k, ldsTotal);
    const unsigned nb = static_cast<unsigned>(ceil_div(a.numSticks - a.stickBegin, lines));
    hipLaunchKernelGGL(k, dim3(nb, 1, batch_dim(b.batch)), dim3(threads), ldsTotal, stream, eng, b, in, values,
                       scale, tw);
    gpu_check_launch("z_forward", stream);
  });
}

template <typename T, typename BT>
void launch_y_backward(const YArgs& a, const BT* in, cx<T>* inter, const cx<T>* tw,
                       hipStream_t stream) {
  if (a.colEnd <= a.colBegin || a.L <= a.zBegin) return;
  with_engine<T, +1, true>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    auto k = a.plainSticks ? y_backward_kernel<decltype(eng), T, BT, true> : y_backward_kernel<decltype(eng), T, BT, false>;
    const std::size_t ldsTotal = lds + col_entries_lds(a, true, y_table<decltype(eng), true>());
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, y_grid(a.colEnd - a.colBegin, ceil_div(a.L - a.zBegin, lines), batch_dim(a.batch)), dim3(threads), ldsTotal, stream, eng, a,
                       in, inter, tw);
    gpu_check_launch("y_backward", stream);
  });
}

template <typename T, typename BT>
void launch_y_forward(const YArgs& a, const cx<T>* inter, BT* out, const cx<T>* tw,
                      hipStream_t stream) {
  if (a.colEnd <= a.colBegin || a.L <= a.zBegin) return;
  with_engine<T, -1, true, !std::is_same<T, float>::value>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    auto k = y_forward_kernel<decltype(eng), T, BT>;
    const std::size_t ldsTotal = lds + col_entries_lds(a, false, y_table<decltype(eng), has_store_pos<decltype(eng)>::value>());
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, y_grid(a.colEnd - a.colBegin, ceil_div(a.L - a.zBegin, lines), batch_dim(a.batch)), dim3(threads), ldsTotal, stream, eng, a,
                       inter, out, tw);
    gpu_check_launch("y_forward", stream);
  });
}

template <typename T>
void launch_x_backward(const XArgs& a, bool r2c, const cx<T>* inter, void* space,
                       const cx<T>* tw, const cx<T>* twHalf, hipStream_t stream) {
  if (a.L <= a.zBegin || a.Y <= 0) return;
  if (r2c && twHalf && a.n % 2 == 0 && a.n >= 4) {
    with_engine<T, +1, true>(a.n / 2, [&](auto eng, int threads, int lines, std::size_t lds) {
      auto k = x_backward_c2r_kernel<decltype(eng), T>;
      const std::size_t ldsTotal =
          lds + std::size_t(lines) * sizeof(cx<T>) + std::size_t(a.n / 2 + 1) * sizeof(int) + 16;
      prepare_kernel(k, ldsTotal);
      hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin, batch_dim(a.batch)), dim3(threads), ldsTotal,
                         stream, eng, a, inter, static_cast<T*>(space), twHalf, tw);
      gpu_check_launch("x_backward_c2r", stream);
    });
    return;
  }
  with_engine<T, +1, true>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    auto k = r2c ? x_backward_kernel<decltype(eng), T, true> : x_backward_kernel<decltype(eng), T, false>;
    const std::size_t ldsTotal = lds + std::size_t(a.n) * sizeof(int) + 16;
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin, batch_dim(a.batch)), dim3(threads), ldsTotal, stream, eng, a,
                       inter, space, tw);
    gpu_check_launch("x_backward", stream);
  });
}

template <typename T>
void launch_x_forward(const XArgs& a, bool r2c, const void* space, cx<T>* inter,
                      const cx<T>* tw, const cx<T>* twHalf, hipStream_t stream) {
  if (a.L <= a.zBegin || a.Y <= 0) return;
  if (r2c && twHalf && a.n % 2 == 0 && a.n >= 4) {
    with_engine<T, -1, false>(a.n / 2, [&](auto eng, int threads, int lines, std::size_t lds) {
      auto k = x_forward_r2c_kernel<decltype(eng), T>;
      const std::size_t ldsTotal = lds + std::size_t(a.n / 2 + 1) * sizeof(int) + 16;
      prepare_kernel(k, ldsTotal);
      hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin, batch_dim(a.batch)), dim3(threads), ldsTotal,
                         stream, eng, a, static_cast<const T*>(space), inter, twHalf, tw);
      gpu_check_launch("x_forward_r2c", stream);
    });
    return;
  }
  with_engine<T, -1, true>(a.n, [&](auto eng, int threads, int lines, std::size_t lds) {
    auto k = r2c ? x_forward_kernel<decltype(eng), T, true> : x_forward_kernel<decltype(eng), T, false>;
    const std::size_t ldsTotal = lds + std::size_t(a.n) * sizeof(int) + 16;
    prepare_kernel(k, ldsTotal);
    hipLaunchKernelGGL(k, dim3(ceil_div(a.Y, lines), a.L - a.zBegin, batch_dim(a.batch)), dim3(threads), ldsTotal, stream, eng, a,
                       space, inter, tw);
    gpu_check_launch("x_forward", stream);
  });
}

}  // namespace dev
}  // namespace spfft
