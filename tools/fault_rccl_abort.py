"""Failure detection on the RCCL plane (run by tests/test_gpu_transform.py with the
testing library): two in-process ranks on one GPU with SPFFT_GPU_EXCHANGE=rccl; fault
injection EXCHANGE_ABORT=2 aborts the communicator at the 2nd exchange. That call and
every later exchange must raise MPIError instead of hanging. Prints ABORT OK."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("SPFFT_AMD_LIBRARY", os.path.join(REPO, "spfft_amd", "_native", "libspfft_amd_testing.so"))
os.environ["SPFFT_GPU_EXCHANGE"] = "rccl"
os.environ["SPFFT_RCCL_SHARE"] = "0"
os.environ["SPFFT_FAULT_EXCHANGE_ABORT"] = "2"


def main():
    import torch
    import spfft_amd as sp
    from spfft_amd.ops._lib import is_testing_library
    from spfft_amd.parallel import make_distributed, run_ranks
    from spfft_amd.utils.indices import sphere_indices

    assert is_testing_library(), "needs libspfft_amd_testing.so"
    dims = (16, 12, 10)
    gidx = sphere_indices(*dims, 0.5)

    def body(rank, comm):
        torch.cuda.set_device(0)
        s = make_distributed(comm, dims, gidx, processing_unit=sp.ProcessingUnit.GPU)
        v = torch.ones(len(s.indices), dtype=torch.complex128, device="cuda")
        s.transform.backward(v)  # exchange 1: fine
        msgs = []
        for _ in range(2):
            try:
                s.transform.forward(None)
                msgs.append(None)
            except sp.MPIError as err:
                msgs.append(str(err))
        return msgs

    for msgs in run_ranks(2, body):
        assert all(m is not None and "abort" in m for m in msgs), msgs
    print("ABORT OK", flush=True)


if __name__ == "__main__":
    main()
