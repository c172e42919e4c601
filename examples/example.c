/* 2x2x2 C2C transform on the host with the C API (SpFFT README example, config 1). */
#include <stdio.h>
#include <stdlib.h>

#include "spfft/spfft.h"

int main(int argc, char** argv) {
  const int dimX = 2, dimY = 2, dimZ = 2;
  const int numValues = dimX * dimY * dimZ;
  int indices[3 * 8];
  double freqValues[2 * 8];
  int i = 0;
  for (int x = 0; x < dimX; ++x)
    for (int y = 0; y < dimY; ++y)
      for (int z = 0; z < dimZ; ++z, ++i) {
        indices[3 * i] = x;
        indices[3 * i + 1] = y;
        indices[3 * i + 2] = z;
        freqValues[2 * i] = i;
        freqValues[2 * i + 1] = -i;
      }

  SpfftGrid grid;
  SpfftError err = spfft_grid_create(&grid, dimX, dimY, dimZ, dimX * dimY, SPFFT_PU_HOST, -1);
  if (err != SPFFT_SUCCESS) exit(err);

  SpfftTransform transform;
  err = spfft_transform_create(&transform, grid, SPFFT_PU_HOST, SPFFT_TRANS_C2C, dimX, dimY, dimZ,
                               dimZ, numValues, SPFFT_INDEX_TRIPLETS, indices);
  if (err != SPFFT_SUCCESS) exit(err);
  /* the transform holds a reference to the grid */
  spfft_grid_destroy(grid);

  err = spfft_transform_backward(transform, freqValues, SPFFT_PU_HOST);
  if (err != SPFFT_SUCCESS) exit(err);
  double* space;
  spfft_transform_get_space_domain(transform, SPFFT_PU_HOST, &space);
  printf("After backward transform:\n");
  for (i = 0; i < numValues; ++i) printf("%f, %f\n", space[2 * i], space[2 * i + 1]);

  err = spfft_transform_forward(transform, SPFFT_PU_HOST, freqValues, SPFFT_FULL_SCALING);
  if (err != SPFFT_SUCCESS) exit(err);
  printf("\nAfter forward transform (with scaling):\n");
  for (i = 0; i < numValues; ++i) printf("%f, %f\n", freqValues[2 * i], freqValues[2 * i + 1]);

  spfft_transform_destroy(transform);
  return 0;
}
