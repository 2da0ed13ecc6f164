"""HBM traffic of the tokenize kernel per launch from rocprofv3 PMC passes.

Usage (GPU box):  python tools/pmc_traffic.py [N] [tag]
Runs two separate `rocprofv3 --kernel-trace --pmc` passes (FETCH_SIZE, WRITE_SIZE -- they do
not fit one pass) over tools/prof_driver.py on the bench workload, then writes
profiles/pmc_traffic.json:  FETCH_SIZE x 2 (the gfx950 correction of MI355X_MICROARCH.md
§HBM) + WRITE_SIZE, KB -> bytes, mean over the dispatches of the first-pass tokenize kernel,
keyed by the sha256 of the kernel sources so bench.py only reports it for the same code.
"""
import csv, glob, hashlib, json, os, re, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = ["dpt_kernels.hip", "dpt_long.hip", "dpt_api.cpp", "dpt_vocab.cpp", "dpt_internal.h"]


def normalized(src: str) -> str:
    """Source text without // comments and whitespace, so comment edits keep the key."""
    return "".join("".join(re.sub(r"//.*", "", line).split()) for line in src.splitlines())


def source_hash(read=None) -> str:
    h = hashlib.sha256()
    for f in SRC:
        if read is None:
            with open(os.path.join(ROOT, "dp-tokenization_amd", "csrc", f)) as fh:
                src = fh.read()
        else:
            src = read(f)
        h.update(normalized(src).encode())
    return h.hexdigest()


def run_pass(counter: str, n: int, out: str, rerun: bool = True, lib: str = None) -> float:
    env = dict(os.environ, TMPDIR="/tmp")
    if lib:
        env["DPT_LIB"] = lib
    cmd = ["rocprofv3", "--kernel-trace", "--pmc", counter, "-d", out, "-o", "run", "--output-format", "csv",
           "--", sys.executable, os.path.join(ROOT, "tools", "prof_driver.py"), str(n), "3", "ascii"]
    if rerun:
        with open(out + ".log", "w") as log:
            subprocess.run(cmd, check=True, stdout=log, stderr=subprocess.STDOUT, env=env, timeout=600)
    vals = []
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if "tokenize_kernel<256" in name and row["Counter_Name"] == counter:   # the first pass only
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise RuntimeError("no %s samples for the tokenize kernel" % counter)
    return sum(vals) / len(vals) * 1024.0   # KB -> bytes


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    tag = sys.argv[2] if len(sys.argv) > 2 else "traffic"
    out = os.path.join(ROOT, "gpurun_out", "pmc_" + tag)
    os.makedirs(out, exist_ok=True)
    rerun = os.environ.get("PMC_REUSE") != "1"   # PMC_REUSE=1: re-read the CSVs of a previous run
    fetch = run_pass("FETCH_SIZE", n, os.path.join(out, "fetch"), rerun)
    write = run_pass("WRITE_SIZE", n, os.path.join(out, "write"), rerun)
    # FETCH_SIZE calibration on THIS kernel's access pattern: the build that stops
    # after prep (-DDPT_STOP=1, `make variant V=stop1`) reads exactly the text (aligned dword buffer loads,
    # n x 256 B) and the offsets (8 (n+1) B) from HBM -- the trie tables stay in L2 -- so known bytes /
    # its raw FETCH_SIZE is the factor for the full kernel's fetches (the guide's x2 is for 16-B streams)
    # (ablibs/ travels to the GPU box; csrc/build/ is in .gpurunignore)
    stop1 = os.path.join(ROOT, "ablibs", "libdpt_stop1.so")
    if not os.path.exists(stop1):
        stop1 = os.path.join(ROOT, "dp-tokenization_amd", "csrc", "build", "var_stop1", "libdpt.so")
    known = n * 256 + 8 * (n + 1)
    factor, cal = 2.0, None
    if os.path.exists(stop1):
        cal = run_pass("FETCH_SIZE", n, os.path.join(out, "fetch_stop1"), rerun, lib=stop1)
        factor = known / cal
    rec = {"source_sha256": source_hash(), "workload": "cfg2 %d x 256 B random ASCII" % n, "n_str": n,
           "fetch_bytes_raw": fetch, "fetch_factor": factor, "fetch_bytes": factor * fetch, "write_bytes": write,
           "traffic_bytes_per_launch": factor * fetch + write,
           "calibration": {"build": "DPT_STOP=1 (prep only)", "known_fetch_bytes": known, "raw_fetch_bytes": cal,
                           "factor": factor} if cal else None,
           "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes); FETCH_SIZE x factor, "
                     "the factor calibrated on the prep-only build of the same kernel (known bytes / raw FETCH_SIZE)"}
    for path in (os.path.join(ROOT, "profiles", "pmc_traffic.json"), os.path.join(out, "pmc_traffic.json")):
        with open(path, "w") as fh:   # the gpurun_out copy is what travels back from a GPU box
            json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
