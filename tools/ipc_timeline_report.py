"""Report of tools/ipc_timeline.sh: per iteration, when each rank's chunk copies ran against the
sending peer's epilogue chunks (host clock shared by the ranks' rocprofv3 traces).

usage: python tools/ipc_timeline_report.py gpurun_out/<tag> [--chunks 8] [--last 3]
"""
import argparse
import csv
import glob
import os


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--chunks", type=int, default=8, help="exchange chunks per iteration (classes / 8)")
    ap.add_argument("--last", type=int, default=3, help="iterations to show")
    a = ap.parse_args()
    ranks = sorted(int(os.path.basename(d)[1:]) for d in glob.glob(os.path.join(a.dir, "r[0-9]*")) if os.path.isdir(d))
    P = len(ranks)
    epi, cps, hot = {}, {}, {}
    for r in ranks:
        kt = glob.glob(os.path.join(a.dir, f"r{r}", "**", "*kernel_trace.csv"), recursive=True)
        mt = glob.glob(os.path.join(a.dir, f"r{r}", "**", "*memory_copy_trace.csv"), recursive=True)
        ks = rows(kt[0])
        epi[r] = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in ks
                        if "k_epilogue_grp" in x["Kernel_Name"])
        hot[r] = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in ks
                        if "k_spmv_hot" in x["Kernel_Name"])
        ms = rows(mt[0]) if mt else []
        d2d = [x for x in ms if "DEVICE_TO_DEVICE" in (x.get("Direction", "") + x.get("Kind", "")).upper()
               or x.get("Source_Agent_Id") == x.get("Destination_Agent_Id")]
        # pulls run as the runtime's blit kernel (PR_OPT_XCHG_IPC_BLIT) appear as kernels, not copies
        blit = [(int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in ks if "copyBuffer" in x["Kernel_Name"]]
        cps[r] = sorted([(int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in d2d] + (blit if not d2d else []))
    t0 = min(v[0][0] for v in epi.values() if v)
    us = lambda t: (t - t0) / 1e3  # noqa: E731
    n_epi = {r: len(epi[r]) for r in ranks}
    print(f"ranks {P}; epilogue dispatches per rank {n_epi}; device copies per rank "
          f"{ {r: len(cps[r]) for r in ranks} }")
    early_total = late_total = 0
    for r in ranks:
        for q in ranks:
            if q == r:
                continue
            per_it_epi = a.chunks if n_epi[q] % a.chunks == 0 and n_epi[q] >= a.chunks * 2 else 1
            it_q = n_epi[q] // per_it_epi
            per_it_cp = (P - 1) * a.chunks
            it_r = len(cps[r]) // per_it_cp
            n = min(a.last, it_q, it_r)
            print(f"\nrank {r} pulling from rank {q} (epilogue launches per iteration on rank {q}: {per_it_epi})")
            for k in range(n, 0, -1):
                e = epi[q][(it_q - k) * per_it_epi:(it_q - k + 1) * per_it_epi]
                c = cps[r][(it_r - k) * per_it_cp:(it_r - k + 1) * per_it_cp]
                last_end = e[-1][1]
                early = sum(1 for s, _ in c if s < last_end)
                early_total += early
                late_total += len(c) - early
                print(f"  iteration -{k}: rank {q} epilogue {us(e[0][0]):10.1f} .. {us(last_end):10.1f} us; "
                      f"rank {r} copies start " + ", ".join(f"{us(s):.1f}" for s, _ in c)
                      + f"  -> {early}/{len(c)} start before the peer's last epilogue chunk ends")
    print(f"\ncopies started before the sender's epilogue ended: {early_total} of {early_total + late_total}")


if __name__ == "__main__":
    main()
