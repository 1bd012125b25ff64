"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes for the dissect
kernel into profiles/pmc_<config>.json (HBM bytes per launch).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are
in KiB; FETCH_SIZE reports exactly half of the bytes of a wide (16 B/lane)
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for
16 B/lane streaming stores (the record store is one dwordx4 per lane)."""
import csv
import json
import sys


def kernel_values(path, counter):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if "dissect_kernel" in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main(fetch_csv, write_csv, out, packets):
    fv = kernel_values(fetch_csv, "FETCH_SIZE")
    wv = kernel_values(write_csv, "WRITE_SIZE")
    f_kib = sum(fv) / len(fv)
    w_kib = sum(wv) / len(wv)
    read_b = 2 * f_kib * 1024
    write_b = w_kib * 1024
    res = {"launches": len(fv), "FETCH_SIZE_KiB": f_kib, "WRITE_SIZE_KiB": w_kib,
           "read_bytes_corrected": read_b, "write_bytes": write_b,
           "hbm_bytes_per_launch": read_b + write_b,
           "bytes_per_packet": (read_b + write_b) / packets,
           "note": "read = 2 x FETCH_SIZE (gfx950 wide-read correction), KiB -> bytes"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]))
