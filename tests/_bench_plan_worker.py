"""One rank of tests/test_multiproc.py::test_bench_multi_gpu_keys_8_ranks: the
multi-GPU keys bench.py puts in its line at N = 8, built by bench.py's own
functions over gloo on CPU (no GPU call in any of them):
  * "config5": bench.config5_plan -- 8,192 requested per rank, agreed over the
    ranks by xdist.gather_seconds, each rank's contiguous range;
  * "rank_devices": xdist.gather_objects of each rank's device (the "PCI
    address" is simulated: rank r on 0000:r:00, one GPU per rank), checked
    distinct by xdist.check_distinct_devices;
  * "xgmi_repair": bench.xgmi_need_plan on rank 0 with 8 GPUs visible, the
    need set from the oracle's GetNeedVects (xrs.go:146-171).
Rank 0 writes the simulated line to OUT_DIR/line.json.

usage: python tests/_bench_plan_worker.py OUT_DIR
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir = sys.argv[1]
    import bench
    from oracle.xrs_oracle import XRS as OracleXRS
    from xrs_amd import dist as xdist

    w = xdist.resolve_world(None)
    xdist.init(w, "gloo")
    plan = bench.config5_plan(8192, 1 << 40, w.rank, w.world,
                              lambda v: xdist.gather_seconds(v, None))
    plans = xdist.gather_objects(plan)
    devs = xdist.gather_objects({"rank": w.rank, "device": w.local,
                                 "pci": f"0000:{w.rank + 0x10:02x}:00"})
    shared = xdist.check_distinct_devices(devs, False)
    if w.rank == 0:
        k = 4
        a_need, b_need = OracleXRS(bench.D, bench.P).get_need_vects(k)
        xg = bench.xgmi_need_plan(0, w.world, k, bench.REC_S, 64, a_need, b_need)
        line = {
            "n_gpus": w.world, "rank_devices": devs, "shared_gpu": shared,
            "config5": {"stripes_total": plan["total"], "stripes_per_rank": plan["n"],
                        "rank_ranges": [[p["first"], p["n"]] for p in plans]},
            "xgmi_repair": {"gpus_visible": w.world, "layouts": xg,
                            "need_set_bytes_remote": xg["half"]["need_set_bytes_remote"]},
        }
        with open(os.path.join(out_dir, "line.json"), "w") as f:
            json.dump(line, f)
    xdist.barrier()
    xdist.finalize()


if __name__ == "__main__":
    main()
