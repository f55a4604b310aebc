"""Copy the evidence of a gpurun_out/<dir> A/B run into profiles/<dest>: each bench log's JSON line (as
.json), the rocprofv3 kernel-stats and SQ/PMC summaries (.csv), pytest tails (.txt).  Raw traces stay in
gpurun_out/ (scratch).   python tools/stash_profile.py gpurun_out/r05_c8b profiles/r05/c8_ab/layouts"""
import glob
import os
import shutil
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    for f in sorted(glob.glob(os.path.join(src, "*"))):
        name = os.path.basename(f)
        if name.endswith(".log") and not name.startswith(("prof_", "sq_")):
            lines = open(f, errors="replace").read().strip().splitlines()
            if name.startswith("pytest"):
                open(os.path.join(dst, name[:-4] + ".txt"), "w").write("\n".join(lines[-3:]) + "\n")
            elif lines and lines[-1].startswith("{"):
                open(os.path.join(dst, name[:-4] + ".json"), "w").write(lines[-1] + "\n")
        elif name.endswith(".csv"):
            shutil.copy(f, os.path.join(dst, name))
    print(dst, sorted(os.listdir(dst)))


if __name__ == "__main__":
    main()
