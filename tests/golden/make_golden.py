#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ from the reference tree.

Runs ONLY in the build container (it reads /root/reference, which does not
exist on the GPU box).  The fixtures it writes are data: numbers parsed from
the reference's own golden output files and the output of the reference's own
coefficient generator (scripts/create_coefficients.py, run as a program).

    python3 tests/golden/make_golden.py [/root/reference]

Outputs
  coefficients.json       create_coefficients.py <p> for p = 1,3,5,7,9:
                          [p][category][poly] = list of (num, den), highest power
                          first (the order fe.h:61-318 stores them)
  reference_outputs.json  parsed numbers from
                          tests/poly_01.output, tests/fe_02_gdm.output,
                          tests/poisson_01_gdm.output, tests/mass_0{1,2}_gdm.output,
                          tests/poisson_02_gdm.mpirun={1,3}.output,
                          applications/wave/tests/*.output,
                          prototypes/cut_poisson_01_gdm.output
"""
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def parse_coefficients(text):
    """Parse the `{{a / b, ...}}` blocks printed by create_coefficients.py."""
    cats = []
    cur = None
    for line in text.splitlines():
        s = line.strip()
        if s == "{{":
            cur = []
        elif "/" in s:
            nums = re.findall(r"(-?\d+\.\d+)\s*/\s*(\d+\.\d+)", s)
            cur.append([[int(float(a)), int(float(b))] for a, b in nums])
        elif s.startswith("}}") and cur is not None:
            cats.append(cur)
            cur = None
    return cats


def blocks(text):
    """Split a deal.II test output into blank-line separated numeric blocks."""
    out, cur = [], []
    for line in text.splitlines():
        if line.strip() == "":
            if cur:
                out.append(cur)
                cur = []
        else:
            cur.append(line)
    if cur:
        out.append(cur)
    return out


def floats(line):
    return [float(x) for x in line.split()]


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    script = os.path.join(ref, "scripts", "create_coefficients.py")

    coeffs = {}
    for p in (1, 3, 5, 7, 9):
        txt = subprocess.run(
            [sys.executable, script, str(p)], capture_output=True, text=True, check=True, timeout=600
        ).stdout
        coeffs[str(p)] = parse_coefficients(txt)
    with open(os.path.join(HERE, "coefficients.json"), "w") as f:
        json.dump({"source": "scripts/create_coefficients.py <p> (run as a program)", "p": coeffs}, f)

    R = {}
    rd = lambda rel: open(os.path.join(ref, rel)).read()

    # tests/poly_01.output: p = 1,3,5,7,9; per category a 21 x (p+1) table
    poly = {}
    bl = blocks(rd("tests/poly_01.output"))
    k = 0
    for p in (1, 3, 5, 7, 9):
        ncat = 1 if p == 1 else p
        poly[str(p)] = [[floats(l) for l in bl[k + c]] for c in range(ncat)]
        k += ncat
    R["poly_01"] = {"source": "tests/poly_01.output", "x": [j / 20 for j in range(21)], "values": poly}

    # tests/fe_02_gdm.output: |value|, |d1|, |d2|, |d3|, |d4| at x=0, interior category
    fe02 = {}
    txt = rd("tests/fe_02_gdm.output")
    for m in re.finditer(r"FESystem<1>\[FE_GDM<1>\((\d+)\)\]:\n((?:\s+[-\d.]+.*\n)+)", txt):
        fe02[m.group(1)] = [floats(l) for l in m.group(2).strip("\n").splitlines()]
    R["fe_02"] = {"source": "tests/fe_02_gdm.output", "abs_values_d0_to_d4": fe02}

    # tests/poisson_01_gdm.output: per p in 1,3,5,7,9: iterations, 11 nodal values, L2 error
    bl = blocks(rd("tests/poisson_01_gdm.output"))
    pois = {}
    for i, p in enumerate((1, 3, 5, 7, 9)):
        its = int(bl[2 * i][0])
        vals = [float(x) for x in bl[2 * i + 1][:-1]]
        err = floats(bl[2 * i + 1][-1])[1]
        pois[str(p)] = {"iterations": its, "values": vals, "l2_error": err}
    R["poisson_01"] = {"source": "tests/poisson_01_gdm.output", "n_subdivisions": 10, "cases": pois}

    R["mass_01"] = {
        "source": "tests/mass_01_gdm.output",
        "error": float(rd("tests/mass_01_gdm.output").split(":")[1]),
    }
    R["mass_02"] = {
        "source": "tests/mass_02_gdm.output",
        "error": float(rd("tests/mass_02_gdm.output").split(":")[1]),
    }

    p02 = {}
    for n in (1, 3):
        bl = blocks(rd("tests/poisson_02_gdm.mpirun=%d.output" % n))
        p02[str(n)] = {
            "dim1": {"iterations": int(bl[0][0]), "values": [float(x) for x in bl[1]]},
            "dim2": {"iterations": int(bl[2][0]), "values": [float(x) for x in bl[3]]},
        }
    R["poisson_02"] = {"source": "tests/poisson_02_gdm.mpirun={1,3}.output", "n_subdivisions": 20, "runs": p02}

    apps = {}
    wdir = os.path.join(ref, "applications/wave/tests")
    for fn in sorted(os.listdir(wdir)):
        if not fn.endswith(".output"):
            continue
        rows, solves = [], []
        for line in open(os.path.join(wdir, fn)):
            s = line.split()
            if len(s) == 5 and re.match(r"^\d+$", s[0]):
                rows.append([int(s[0])] + [float(x) for x in s[1:]])
            m = re.search(r"solved in (\d+)", line)
            if m:
                solves.append(int(m.group(1)))
        cfg = json.load(open(os.path.join(wdir, fn.replace(".output", ".json"))))
        apps[fn.replace(".output", "")] = {"config": cfg, "steps": rows, "cg_iterations": solves}
    R["wave_app"] = {"source": "applications/wave/tests/*.output", "cases": apps}

    txt = rd("prototypes/cut_poisson_01_gdm.output")
    R["cut_poisson_01"] = {"source": "prototypes/cut_poisson_01_gdm.output", "text": txt.splitlines()}

    # applications/advection/tests/test_01.output: advection-convergence.cc's
    # "parallel-ramp-degree" ConvergenceTable (two blocks, p = 3 and 5)
    txt = rd("applications/advection/tests/test_01.output")
    header, rows = None, []
    for line in txt.splitlines():
        s = line.split()
        if not s:
            continue
        if s[0] == "fe_degree":
            header = s
        else:
            rows.append([int(s[0]), float(s[1]), int(s[2])] + [float(x) for x in s[3:]])
    R["advection_test_01"] = {"source": "applications/advection/tests/test_01.output", "columns": header,
                              "rows": rows, "text": txt.splitlines()}

    with open(os.path.join(HERE, "reference_outputs.json"), "w") as f:
        json.dump(R, f, indent=1)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
