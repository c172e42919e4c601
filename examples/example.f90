! 2x2x2 C2C transform on the host from Fortran (SpFFT README example, config 1).
program main
  use iso_c_binding
  use spfft
  implicit none
  integer :: i, j, k, counter
  integer, parameter :: dimX = 2, dimY = 2, dimZ = 2
  integer, parameter :: maxNumLocalZColumns = dimX * dimY
  integer, parameter :: processingUnit = SPFFT_PU_HOST
  integer, parameter :: maxNumThreads = -1
  type(c_ptr) :: grid = c_null_ptr
  type(c_ptr) :: transform = c_null_ptr
  integer :: errorCode = 0
  integer, dimension(dimX * dimY * dimZ * 3), target :: indices = 0
  complex(c_double), dimension(dimX * dimY * dimZ), target :: freqValues
  complex(c_double), pointer :: spaceDomain(:, :, :)
  type(c_ptr) :: realValuesPtr

  counter = 0
  do k = 1, dimZ
    do j = 1, dimY
      do i = 1, dimX
        freqValues(counter + 1) = cmplx(counter, -counter, kind=c_double)
        indices(counter * 3 + 1) = i - 1
        indices(counter * 3 + 2) = j - 1
        indices(counter * 3 + 3) = k - 1
        counter = counter + 1
      end do
    end do
  end do

  errorCode = spfft_grid_create(grid, dimX, dimY, dimZ, maxNumLocalZColumns, processingUnit, &
                                maxNumThreads)
  if (errorCode /= SPFFT_SUCCESS) error stop

  errorCode = spfft_transform_create(transform, grid, processingUnit, SPFFT_TRANS_C2C, dimX, dimY, &
                                     dimZ, dimZ, size(freqValues), SPFFT_INDEX_TRIPLETS, indices)
  if (errorCode /= SPFFT_SUCCESS) error stop

  ! the transform keeps the grid alive
  errorCode = spfft_grid_destroy(grid)
  if (errorCode /= SPFFT_SUCCESS) error stop

  errorCode = spfft_transform_backward(transform, c_loc(freqValues), processingUnit)
  if (errorCode /= SPFFT_SUCCESS) error stop

  errorCode = spfft_transform_get_space_domain(transform, processingUnit, realValuesPtr)
  if (errorCode /= SPFFT_SUCCESS) error stop
  call c_f_pointer(realValuesPtr, spaceDomain, [dimX, dimY, dimZ])

  print *, "After backward transform:"
  do k = 1, dimZ
    do j = 1, dimY
      do i = 1, dimX
        print *, spaceDomain(i, j, k)
      end do
    end do
  end do

  ! forward transform (may overwrite the space domain)
  errorCode = spfft_transform_forward(transform, processingUnit, c_loc(freqValues), &
                                      SPFFT_FULL_SCALING)
  if (errorCode /= SPFFT_SUCCESS) error stop

  print *, "After forward transform (with scaling):"
  do i = 1, size(freqValues)
    print *, freqValues(i)
  end do

  errorCode = spfft_transform_destroy(transform)
  if (errorCode /= SPFFT_SUCCESS) error stop
end program
