"""The persistent kernels' launches in a rocprofv3 kernel trace (run_kernel_trace.csv), in order:
one CSV row per launch of k_onchip / k_resident / k_wave / k_solo (kernel, grid, VGPRs, duration in
microseconds), to set beside bench.py's HIP-event `mean_launch_us` of the same command.

usage: python scripts/rocprof_launches.py <run_kernel_trace.csv> > profiles/<round>_rocprof_timed_launches.csv
"""
import csv
import re
import sys

KERNELS = re.compile(r"(k_onchip<[^>]*>|k_resident<[^>]*>|k_wave<[^>]*>|k_solo\w*<[^>]*>)")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "vgpr", "agpr", "lds_bytes", "duration_us"])
    for r in rows:
        mt = KERNELS.search(r["Kernel_Name"])
        if mt is None:
            continue
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        w.writerow([mt.group(1), r["Grid_Size_X"], r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"],
                    f"{dur:.1f}"])


if __name__ == "__main__":
    main()
