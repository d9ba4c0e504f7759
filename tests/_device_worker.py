"""One rank of tests/test_multiproc.py's device-identity tests: the gather of
every rank's GPU identity and the one-rank-per-GPU check bench.py runs at
start-up (xrs_amd.dist.gather_objects / check_distinct_devices), over gloo on
CPU.  Each rank's "PCI address" comes from XRS_TEST_PCI (comma-separated,
indexed by rank), standing in for torch.cuda.get_device_properties.

usage: python tests/_device_worker.py OUT_DIR
exit status 3: the check refused the layout (as bench.py does).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir = sys.argv[1]
    from xrs_amd import dist as xdist

    w = xdist.resolve_world(None)
    xdist.init(w, "gloo")
    pci = os.environ["XRS_TEST_PCI"].split(",")[w.rank]
    devs = xdist.gather_objects({"rank": w.rank, "device": 0, "pci": pci})
    try:
        shared = xdist.check_distinct_devices(devs, xdist.rehearsal_env())
    except xdist.SharedDevice as e:
        if w.rank == 0:
            with open(os.path.join(out_dir, "refused.txt"), "w") as f:
                f.write(str(e))
        else:  # let rank 0 write first (launch_local stops the rest on a failure)
            import time
            time.sleep(2)
        sys.exit(3)
    if w.rank == 0:
        with open(os.path.join(out_dir, "result.json"), "w") as f:
            json.dump({"devices": devs, "shared": shared}, f)
    xdist.barrier()
    xdist.finalize()


if __name__ == "__main__":
    main()
