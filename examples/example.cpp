// 2x2x2 C2C transform on the host with the C++ API (SpFFT README example, config 1).
#include <complex>
#include <iostream>
#include <vector>

#include "spfft/spfft.hpp"

int main() {
  const int dimX = 2, dimY = 2, dimZ = 2;
  std::cout << "Dimensions: x = " << dimX << ", y = " << dimY << ", z = " << dimZ << "\n\n";

  // all frequency triplets (x, y, z); values in the same order
  std::vector<int> indices;
  for (int x = 0; x < dimX; ++x)
    for (int y = 0; y < dimY; ++y)
      for (int z = 0; z < dimZ; ++z) indices.insert(indices.end(), {x, y, z});
  const int numValues = static_cast<int>(indices.size() / 3);
  std::vector<std::complex<double>> freqValues;
  for (int i = 0; i < numValues; ++i) freqValues.emplace_back(i, -i);

  std::cout << "Input:\n";
  for (const auto& v : freqValues) std::cout << v.real() << ", " << v.imag() << "\n";

  // grid for transforms up to 2x2x2 with 4 z-sticks, host only, default threads
  spfft::Grid grid(dimX, dimY, dimZ, dimX * dimY, SPFFT_PU_HOST, -1);
  auto transform = grid.create_transform(SPFFT_PU_HOST, SPFFT_TRANS_C2C, dimX, dimY, dimZ, dimZ,
                                         numValues, SPFFT_INDEX_TRIPLETS, indices.data());

  transform.backward(reinterpret_cast<double*>(freqValues.data()), SPFFT_PU_HOST);
  auto* space = reinterpret_cast<std::complex<double>*>(transform.space_domain_data(SPFFT_PU_HOST));
  std::cout << "\nAfter backward transform:\n";
  for (int i = 0; i < transform.local_slice_size(); ++i)
    std::cout << space[i].real() << ", " << space[i].imag() << "\n";

  transform.forward(SPFFT_PU_HOST, reinterpret_cast<double*>(freqValues.data()), SPFFT_FULL_SCALING);
  std::cout << "\nAfter forward transform (with scaling):\n";
  for (const auto& v : freqValues) std::cout << v.real() << ", " << v.imag() << "\n";
  return 0;
}
