"""Node-local shared-memory collectives (the relay data plane's host synchronisation)
against the torch.distributed gloo control plane, one OS process per rank:
    python -m torch.distributed.run --standalone --local-addr=127.0.0.1 --nproc-per-node=3 \
        tools/shm_probe.py [--iters N]
Prints one line per rank: "SHM OK rank=r shm_us=... comm_us=...".
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
# the probe lives in the testing library (not in the release ABI)
os.environ.setdefault("SPFFT_AMD_LIBRARY", os.path.join(REPO, "spfft_amd", "_native", "libspfft_amd_testing.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    args = ap.parse_args()
    import torch.distributed as dist
    from spfft_amd.parallel.comm import TorchDistComm

    dist.init_process_group("gloo")
    comm = TorchDistComm()
    try:
        shm, com = comm.shm_check(args.iters)
    except Exception as e:  # noqa: BLE001
        # (fault injection SHM_EXIT: a peer left; the wait must end with an error)
        print(f"SHM ERROR rank={dist.get_rank()} {e}", flush=True)
        os._exit(0)
    print(f"SHM OK rank={dist.get_rank()} " + json.dumps({"shm_us": shm, "comm_us": com}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
