! SpFFT-AMD Fortran module: iso_c_binding interfaces to the C API (spfft/spfft.h).
! Constants mirror spfft/types.h and spfft/errors.h (reference: include/spfft/spfft.f90).
! Data arguments are type(c_ptr), so host arrays (c_loc) and device pointers both work.
! Distributed grids take the communicator as a Fortran integer (MPI_Comm_f2c shims).
module spfft
  use iso_c_binding
  implicit none

  integer(c_int), parameter :: SPFFT_EXCH_DEFAULT = 0
  integer(c_int), parameter :: SPFFT_EXCH_BUFFERED = 1
  integer(c_int), parameter :: SPFFT_EXCH_BUFFERED_FLOAT = 2
  integer(c_int), parameter :: SPFFT_EXCH_COMPACT_BUFFERED = 3
  integer(c_int), parameter :: SPFFT_EXCH_COMPACT_BUFFERED_FLOAT = 4
  integer(c_int), parameter :: SPFFT_EXCH_UNBUFFERED = 5
  integer(c_int), parameter :: SPFFT_PU_HOST = 1
  integer(c_int), parameter :: SPFFT_PU_GPU = 2
  integer(c_int), parameter :: SPFFT_INDEX_TRIPLETS = 0
  integer(c_int), parameter :: SPFFT_TRANS_C2C = 0
  integer(c_int), parameter :: SPFFT_TRANS_R2C = 1
  integer(c_int), parameter :: SPFFT_NO_SCALING = 0
  integer(c_int), parameter :: SPFFT_FULL_SCALING = 1
  integer(c_int), parameter :: SPFFT_SUCCESS = 0
  integer(c_int), parameter :: SPFFT_UNKNOWN_ERROR = 1
  integer(c_int), parameter :: SPFFT_INVALID_HANDLE_ERROR = 2
  integer(c_int), parameter :: SPFFT_OVERFLOW_ERROR = 3
  integer(c_int), parameter :: SPFFT_ALLOCATION_ERROR = 4
  integer(c_int), parameter :: SPFFT_INVALID_PARAMETER_ERROR = 5
  integer(c_int), parameter :: SPFFT_DUPLICATE_INDICES_ERROR = 6
  integer(c_int), parameter :: SPFFT_INVALID_INDICES_ERROR = 7
  integer(c_int), parameter :: SPFFT_MPI_SUPPORT_ERROR = 8
  integer(c_int), parameter :: SPFFT_MPI_ERROR = 9
  integer(c_int), parameter :: SPFFT_MPI_PARAMETER_MISMATCH_ERROR = 10
  integer(c_int), parameter :: SPFFT_HOST_EXECUTION_ERROR = 11
  integer(c_int), parameter :: SPFFT_FFTW_ERROR = 12
  integer(c_int), parameter :: SPFFT_GPU_ERROR = 13
  integer(c_int), parameter :: SPFFT_GPU_PRECEDING_ERROR = 14
  integer(c_int), parameter :: SPFFT_GPU_SUPPORT_ERROR = 15
  integer(c_int), parameter :: SPFFT_GPU_ALLOCATION_ERROR = 16
  integer(c_int), parameter :: SPFFT_GPU_LAUNCH_ERROR = 17
  integer(c_int), parameter :: SPFFT_GPU_NO_DEVICE_ERROR = 18
  integer(c_int), parameter :: SPFFT_GPU_INVALID_VALUE_ERROR = 19
  integer(c_int), parameter :: SPFFT_GPU_INVALID_DEVICE_PTR_ERROR = 20
  integer(c_int), parameter :: SPFFT_GPU_COPY_ERROR = 21
  integer(c_int), parameter :: SPFFT_GPU_FFT_ERROR = 22
  integer(c_int), parameter :: SPFFT_INTERNAL_ERROR = 23

  interface
    integer(c_int) function spfft_grid_create(grid, maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, processingUnit, maxNumThreads) bind(C, name='spfft_grid_create')
      use iso_c_binding
      type(c_ptr), intent(out) :: grid
      integer(c_int), value :: maxDimX
      integer(c_int), value :: maxDimY
      integer(c_int), value :: maxDimZ
      integer(c_int), value :: maxNumLocalZColumns
      integer(c_int), value :: processingUnit
      integer(c_int), value :: maxNumThreads
    end function spfft_grid_create

    integer(c_int) function spfft_grid_create_distributed(grid, maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxLocalZLength, processingUnit, maxNumThreads, comm, exchangeType) bind(C, name='spfft_grid_create_distributed_fortran')
      use iso_c_binding
      type(c_ptr), intent(out) :: grid
      integer(c_int), value :: maxDimX
      integer(c_int), value :: maxDimY
      integer(c_int), value :: maxDimZ
      integer(c_int), value :: maxNumLocalZColumns
      integer(c_int), value :: maxLocalZLength
      integer(c_int), value :: processingUnit
      integer(c_int), value :: maxNumThreads
      integer(c_int), value :: comm
      integer(c_int), value :: exchangeType
    end function spfft_grid_create_distributed

    integer(c_int) function spfft_grid_destroy(grid) bind(C, name='spfft_grid_destroy')
      use iso_c_binding
      type(c_ptr), value :: grid
    end function spfft_grid_destroy

    integer(c_int) function spfft_grid_max_dim_x(grid, val) bind(C, name='spfft_grid_max_dim_x')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_grid_max_dim_x

    integer(c_int) function spfft_grid_max_dim_y(grid, val) bind(C, name='spfft_grid_max_dim_y')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_grid_max_dim_y

    integer(c_int) function spfft_grid_max_dim_z(grid, val) bind(C, name='spfft_grid_max_dim_z')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_grid_max_dim_z

    integer(c_int) function spfft_grid_max_num_local_z_columns(grid, val) bind(C, name='spfft_grid_max_num_local_z_columns')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_grid_max_num_local_z_columns

    integer(c_int) function spfft_grid_max_local_z_length(grid, val) bind(C, name='spfft_grid_max_local_z_length')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_grid_max_local_z_length

    integer(c_int) function spfft_grid_processing_unit(grid, val) bind(C, name='spfft_grid_processing_unit')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_grid_processing_unit

    integer(c_int) function spfft_grid_device_id(grid, val) bind(C, name='spfft_grid_device_id')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_grid_device_id

    integer(c_int) function spfft_grid_num_threads(grid, val) bind(C, name='spfft_grid_num_threads')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_grid_num_threads

    integer(c_int) function spfft_grid_communicator(grid, comm) bind(C, name='spfft_grid_communicator_fortran')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: comm
    end function spfft_grid_communicator

    integer(c_int) function spfft_transform_create(transform, grid, processingUnit, transformType, dimX, dimY, dimZ, localZLength, numLocalElements, indexFormat, indices) bind(C, name='spfft_transform_create')
      use iso_c_binding
      type(c_ptr), intent(out) :: transform
      type(c_ptr), value :: grid
      integer(c_int), value :: processingUnit
      integer(c_int), value :: transformType
      integer(c_int), value :: dimX
      integer(c_int), value :: dimY
      integer(c_int), value :: dimZ
      integer(c_int), value :: localZLength
      integer(c_int), value :: numLocalElements
      integer(c_int), value :: indexFormat
      integer(c_int), dimension(*) :: indices
    end function spfft_transform_create

    integer(c_int) function spfft_transform_destroy(transform) bind(C, name='spfft_transform_destroy')
      use iso_c_binding
      type(c_ptr), value :: transform
    end function spfft_transform_destroy

    integer(c_int) function spfft_transform_clone(transform, newTransform) bind(C, name='spfft_transform_clone')
      use iso_c_binding
      type(c_ptr), value :: transform
      type(c_ptr), intent(out) :: newTransform
    end function spfft_transform_clone

    integer(c_int) function spfft_transform_forward(transform, inputLocation, output, scaling) bind(C, name='spfft_transform_forward')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), value :: inputLocation
      type(c_ptr), value :: output
      integer(c_int), value :: scaling
    end function spfft_transform_forward

    integer(c_int) function spfft_transform_backward(transform, input, outputLocation) bind(C, name='spfft_transform_backward')
      use iso_c_binding
      type(c_ptr), value :: transform
      type(c_ptr), value :: input
      integer(c_int), value :: outputLocation
    end function spfft_transform_backward

    integer(c_int) function spfft_transform_get_space_domain(transform, dataLocation, dataPtr) bind(C, name='spfft_transform_get_space_domain')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), value :: dataLocation
      type(c_ptr), intent(out) :: dataPtr
    end function spfft_transform_get_space_domain

    integer(c_int) function spfft_transform_dim_x(transform, val) bind(C, name='spfft_transform_dim_x')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_transform_dim_x

    integer(c_int) function spfft_transform_dim_y(transform, val) bind(C, name='spfft_transform_dim_y')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_transform_dim_y

    integer(c_int) function spfft_transform_dim_z(transform, val) bind(C, name='spfft_transform_dim_z')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_transform_dim_z

    integer(c_int) function spfft_transform_local_z_length(transform, val) bind(C, name='spfft_transform_local_z_length')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_transform_local_z_length

    integer(c_int) function spfft_transform_local_slice_size(transform, val) bind(C, name='spfft_transform_local_slice_size')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_transform_local_slice_size

    integer(c_int) function spfft_transform_local_z_offset(transform, val) bind(C, name='spfft_transform_local_z_offset')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_transform_local_z_offset

    integer(c_int) function spfft_transform_num_local_elements(transform, val) bind(C, name='spfft_transform_num_local_elements')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_transform_num_local_elements

    integer(c_int) function spfft_transform_device_id(transform, val) bind(C, name='spfft_transform_device_id')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_transform_device_id

    integer(c_int) function spfft_transform_num_threads(transform, val) bind(C, name='spfft_transform_num_threads')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_transform_num_threads

    integer(c_int) function spfft_transform_global_size(transform, val) bind(C, name='spfft_transform_global_size')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_long_long), intent(out) :: val
    end function spfft_transform_global_size

    integer(c_int) function spfft_transform_num_global_elements(transform, val) bind(C, name='spfft_transform_num_global_elements')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_long_long), intent(out) :: val
    end function spfft_transform_num_global_elements

    integer(c_int) function spfft_transform_communicator(transform, comm) bind(C, name='spfft_transform_communicator_fortran')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: comm
    end function spfft_transform_communicator

    integer(c_int) function spfft_multi_transform_forward(numTransforms, transforms, inputLocations, outputPointers, scalingTypes) bind(C, name='spfft_multi_transform_forward')
      use iso_c_binding
      integer(c_int), value :: numTransforms
      type(c_ptr), dimension(*) :: transforms
      integer(c_int), dimension(*) :: inputLocations
      type(c_ptr), dimension(*) :: outputPointers
      integer(c_int), dimension(*) :: scalingTypes
    end function spfft_multi_transform_forward

    integer(c_int) function spfft_multi_transform_backward(numTransforms, transforms, inputPointers, outputLocations) bind(C, name='spfft_multi_transform_backward')
      use iso_c_binding
      integer(c_int), value :: numTransforms
      type(c_ptr), dimension(*) :: transforms
      type(c_ptr), dimension(*) :: inputPointers
      integer(c_int), dimension(*) :: outputLocations
    end function spfft_multi_transform_backward

    integer(c_int) function spfft_float_grid_create(grid, maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, processingUnit, maxNumThreads) bind(C, name='spfft_float_grid_create')
      use iso_c_binding
      type(c_ptr), intent(out) :: grid
      integer(c_int), value :: maxDimX
      integer(c_int), value :: maxDimY
      integer(c_int), value :: maxDimZ
      integer(c_int), value :: maxNumLocalZColumns
      integer(c_int), value :: processingUnit
      integer(c_int), value :: maxNumThreads
    end function spfft_float_grid_create

    integer(c_int) function spfft_float_grid_create_distributed(grid, maxDimX, maxDimY, maxDimZ, maxNumLocalZColumns, maxLocalZLength, processingUnit, maxNumThreads, comm, exchangeType) bind(C, name='spfft_float_grid_create_distributed_fortran')
      use iso_c_binding
      type(c_ptr), intent(out) :: grid
      integer(c_int), value :: maxDimX
      integer(c_int), value :: maxDimY
      integer(c_int), value :: maxDimZ
      integer(c_int), value :: maxNumLocalZColumns
      integer(c_int), value :: maxLocalZLength
      integer(c_int), value :: processingUnit
      integer(c_int), value :: maxNumThreads
      integer(c_int), value :: comm
      integer(c_int), value :: exchangeType
    end function spfft_float_grid_create_distributed

    integer(c_int) function spfft_float_grid_destroy(grid) bind(C, name='spfft_float_grid_destroy')
      use iso_c_binding
      type(c_ptr), value :: grid
    end function spfft_float_grid_destroy

    integer(c_int) function spfft_float_grid_max_dim_x(grid, val) bind(C, name='spfft_float_grid_max_dim_x')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_float_grid_max_dim_x

    integer(c_int) function spfft_float_grid_max_dim_y(grid, val) bind(C, name='spfft_float_grid_max_dim_y')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_float_grid_max_dim_y

    integer(c_int) function spfft_float_grid_max_dim_z(grid, val) bind(C, name='spfft_float_grid_max_dim_z')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_float_grid_max_dim_z

    integer(c_int) function spfft_float_grid_max_num_local_z_columns(grid, val) bind(C, name='spfft_float_grid_max_num_local_z_columns')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_float_grid_max_num_local_z_columns

    integer(c_int) function spfft_float_grid_max_local_z_length(grid, val) bind(C, name='spfft_float_grid_max_local_z_length')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_float_grid_max_local_z_length

    integer(c_int) function spfft_float_grid_processing_unit(grid, val) bind(C, name='spfft_float_grid_processing_unit')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_float_grid_processing_unit

    integer(c_int) function spfft_float_grid_device_id(grid, val) bind(C, name='spfft_float_grid_device_id')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_float_grid_device_id

    integer(c_int) function spfft_float_grid_num_threads(grid, val) bind(C, name='spfft_float_grid_num_threads')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: val
    end function spfft_float_grid_num_threads

    integer(c_int) function spfft_float_grid_communicator(grid, comm) bind(C, name='spfft_float_grid_communicator_fortran')
      use iso_c_binding
      type(c_ptr), value :: grid
      integer(c_int), intent(out) :: comm
    end function spfft_float_grid_communicator

    integer(c_int) function spfft_float_transform_create(transform, grid, processingUnit, transformType, dimX, dimY, dimZ, localZLength, numLocalElements, indexFormat, indices) bind(C, name='spfft_float_transform_create')
      use iso_c_binding
      type(c_ptr), intent(out) :: transform
      type(c_ptr), value :: grid
      integer(c_int), value :: processingUnit
      integer(c_int), value :: transformType
      integer(c_int), value :: dimX
      integer(c_int), value :: dimY
      integer(c_int), value :: dimZ
      integer(c_int), value :: localZLength
      integer(c_int), value :: numLocalElements
      integer(c_int), value :: indexFormat
      integer(c_int), dimension(*) :: indices
    end function spfft_float_transform_create

    integer(c_int) function spfft_float_transform_destroy(transform) bind(C, name='spfft_float_transform_destroy')
      use iso_c_binding
      type(c_ptr), value :: transform
    end function spfft_float_transform_destroy

    integer(c_int) function spfft_float_transform_clone(transform, newTransform) bind(C, name='spfft_float_transform_clone')
      use iso_c_binding
      type(c_ptr), value :: transform
      type(c_ptr), intent(out) :: newTransform
    end function spfft_float_transform_clone

    integer(c_int) function spfft_float_transform_forward(transform, inputLocation, output, scaling) bind(C, name='spfft_float_transform_forward')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), value :: inputLocation
      type(c_ptr), value :: output
      integer(c_int), value :: scaling
    end function spfft_float_transform_forward

    integer(c_int) function spfft_float_transform_backward(transform, input, outputLocation) bind(C, name='spfft_float_transform_backward')
      use iso_c_binding
      type(c_ptr), value :: transform
      type(c_ptr), value :: input
      integer(c_int), value :: outputLocation
    end function spfft_float_transform_backward

    integer(c_int) function spfft_float_transform_get_space_domain(transform, dataLocation, dataPtr) bind(C, name='spfft_float_transform_get_space_domain')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), value :: dataLocation
      type(c_ptr), intent(out) :: dataPtr
    end function spfft_float_transform_get_space_domain

    integer(c_int) function spfft_float_transform_dim_x(transform, val) bind(C, name='spfft_float_transform_dim_x')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_float_transform_dim_x

    integer(c_int) function spfft_float_transform_dim_y(transform, val) bind(C, name='spfft_float_transform_dim_y')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_float_transform_dim_y

    integer(c_int) function spfft_float_transform_dim_z(transform, val) bind(C, name='spfft_float_transform_dim_z')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_float_transform_dim_z

    integer(c_int) function spfft_float_transform_local_z_length(transform, val) bind(C, name='spfft_float_transform_local_z_length')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_float_transform_local_z_length

    integer(c_int) function spfft_float_transform_local_slice_size(transform, val) bind(C, name='spfft_float_transform_local_slice_size')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_float_transform_local_slice_size

    integer(c_int) function spfft_float_transform_local_z_offset(transform, val) bind(C, name='spfft_float_transform_local_z_offset')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_float_transform_local_z_offset

    integer(c_int) function spfft_float_transform_num_local_elements(transform, val) bind(C, name='spfft_float_transform_num_local_elements')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_float_transform_num_local_elements

    integer(c_int) function spfft_float_transform_device_id(transform, val) bind(C, name='spfft_float_transform_device_id')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_float_transform_device_id

    integer(c_int) function spfft_float_transform_num_threads(transform, val) bind(C, name='spfft_float_transform_num_threads')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: val
    end function spfft_float_transform_num_threads

    integer(c_int) function spfft_float_transform_global_size(transform, val) bind(C, name='spfft_float_transform_global_size')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_long_long), intent(out) :: val
    end function spfft_float_transform_global_size

    integer(c_int) function spfft_float_transform_num_global_elements(transform, val) bind(C, name='spfft_float_transform_num_global_elements')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_long_long), intent(out) :: val
    end function spfft_float_transform_num_global_elements

    integer(c_int) function spfft_float_transform_communicator(transform, comm) bind(C, name='spfft_float_transform_communicator_fortran')
      use iso_c_binding
      type(c_ptr), value :: transform
      integer(c_int), intent(out) :: comm
    end function spfft_float_transform_communicator

    integer(c_int) function spfft_float_multi_transform_forward(numTransforms, transforms, inputLocations, outputPointers, scalingTypes) bind(C, name='spfft_float_multi_transform_forward')
      use iso_c_binding
      integer(c_int), value :: numTransforms
      type(c_ptr), dimension(*) :: transforms
      integer(c_int), dimension(*) :: inputLocations
      type(c_ptr), dimension(*) :: outputPointers
      integer(c_int), dimension(*) :: scalingTypes
    end function spfft_float_multi_transform_forward

    integer(c_int) function spfft_float_multi_transform_backward(numTransforms, transforms, inputPointers, outputLocations) bind(C, name='spfft_float_multi_transform_backward')
      use iso_c_binding
      integer(c_int), value :: numTransforms
      type(c_ptr), dimension(*) :: transforms
      type(c_ptr), dimension(*) :: inputPointers
      integer(c_int), dimension(*) :: outputLocations
    end function spfft_float_multi_transform_backward

  end interface
end module spfft
