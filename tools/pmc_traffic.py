"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes per kernel.

gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE = TCC_EA0_RDREQ x 64 B reads
exactly 1/2 of the bytes of a wide (16 B/lane) coalesced streaming read; for other access
widths it is uncalibrated.  `hbm_bytes_per_launch` applies the guide's gfx950 correction
(2 x FETCH_SIZE + WRITE_SIZE, KB x 1024); the raw sum is kept as `hbm_bytes_per_launch_raw`
(our kernels also use 4-B loads, for which the factor is uncalibrated: the two bracket it).

    python tools/pmc_traffic.py <dir with *_counter_collection.csv>
"""
import collections
import csv
import glob
import json
import os
import sys

# first match wins: the specific kernel names before the op names they are templated on
NAMES = {"lse_bound_kernel": "gmm_estep_bound", "lse_fixup_kernel": "gmm_estep_fixup",
         "OpGmmE<3, true>, 2, true>": "gmm_estep_hinted",
         "lse_finalize": "lse_finalize",
         "sym_fwd_pkn_kernelILi3ELb1ELi3": "ode_self_fwd_sym6", "sym_fwd_pkn_kernelILi3ELb1ELi4": "ode_self_fwd_sym8",
         "sym_fwd_pkn_kernel": "ode_self_fwd_symN",
         "sym_fwd_pk8_kernel": "ode_self_fwd_sym8", "scx_kernel": "sym_centred_reduction",
         "scx_merge": "sym_centred_merge", "sym_fwd_pk_kernel": "ode_self_fwd_sym", "sym_fwd_kernel": "ode_self_fwd_sym",
         "sym_fwd_pk4_kernel": "ode_self_fwd_sym4", "sym_fwd4_merge": "sym_fwd_merge",
         "sym_bwd_pk4_kernel": "ode_self_bwd", "sym_bwd_pk_kernel": "ode_self_bwd", "sym_bwd_kernel": "ode_self_bwd", "sym_merge_kernel": "sym_merge",
         "OpOdeSelfBwd": "ode_self_bwd_ordered", "OpOdeSelfFwd": "ode_self_fwd",
         "OpGmmE": "gmm_estep", "OpGmmM": "gmm_mstep", "OpGmmTargets": "gmm_targets",
         "merge_slabs": "merge_slabs",
         "cx_kernel": "centred_reduction"}


def short(kname):
    for k, v in NAMES.items():
        if k in kname:
            return v
    return None


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            s = short(r["Kernel_Name"])
            if s is None:
                continue
            acc[s][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, c in acc.items():
        fetch = sum(c.get("FETCH_SIZE", [0])) / max(1, len(c.get("FETCH_SIZE", [1])))
        write = sum(c.get("WRITE_SIZE", [0])) / max(1, len(c.get("WRITE_SIZE", [1])))
        out[k] = {"fetch_kb_per_launch": fetch, "write_kb_per_launch": write,
                  "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
                  "hbm_bytes_per_launch_raw": (fetch + write) * 1024,
                  "launches": len(c.get("FETCH_SIZE", c.get("WRITE_SIZE", [])))}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
