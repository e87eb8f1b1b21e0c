"""The `odesat` command line (odesat_amd/csrc/cli.cpp; the reference's src/main.rs:12-397).

CPU: argument handling (clap's required flags, bad values, stoch's restricted flags) -- no solver is
created on those paths.  GPU: solve / batch / inter / stoch end to end on small formulas, the
reported assignment re-checked on the host against the file's clauses."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "odesat_amd", "bin", "odesat")


def run(*args, timeout=120):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} is not built (make -C odesat_amd/csrc)")
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=timeout)


def planted(tmp_path, n=60, m=240, seed=3):
    """A satisfiable random 3-SAT formula: every clause agrees with a hidden assignment."""
    rng = np.random.default_rng(seed)
    hidden = rng.integers(0, 2, n).astype(bool)
    lines = [f"p cnf {n} {m}"]
    while len(lines) <= m:
        vs = rng.choice(n, 3, replace=False)
        sg = rng.integers(0, 2, 3).astype(bool)
        if any(hidden[v] != s for v, s in zip(vs, sg)):  # some literal is true under `hidden`
            lines.append(" ".join(str(-(v + 1) if s else v + 1) for v, s in zip(vs, sg)) + " 0")
    p = tmp_path / "planted.cnf"
    p.write_text("\n".join(lines) + "\n")
    return p, lines[1:]


def parse_render(text):
    out = {}
    for line in text.strip().splitlines():
        a, b = line.split()
        out[int(a)] = b == "1"
    return out


def satisfies(assign, clause_lines):
    for ln in clause_lines:
        lits = [int(t) for t in ln.split()[:-1]]
        if not any(assign.get(abs(x), False) != (x < 0) for x in lits):
            return False
    return True


# ------------------------------------------------------------------------------------------ CPU
def test_help():
    r = run("--help")
    assert r.returncode == 0
    for cmd in ("solve", "batch", "inter", "--step-size", "--batch-size"):
        assert cmd in r.stdout


@pytest.mark.parametrize("argv,needle", [
    ((), "subcommand"),
    (("frobnicate",), "unrecognized subcommand"),
    (("solve",), "--input"),
    (("batch", "-f", "x.cnf", "-b", "4"), "--step-number"),
    (("inter", "-f", "x.cnf"), "--batch-size"),
    (("solve", "-f", "x.cnf", "-s", "abc"), "invalid value"),
    (("batch", "-f", "x.cnf", "-n", "-5", "-b", "2"), "invalid value"),
    (("solve", "-f", "x.cnf", "--bogus", "1"), "unexpected argument"),
    (("stoch", "-f", "x.cnf", "-s", "0.1"), "stoch takes only"),
    (("solve", "-f"), "value is required"),
    (("inter", "-f", "x.cnf", "-b", "0"), "batch-size"),
    (("solve", "-f", "x.cnf", "--run-chunk", "0"), "--run-chunk"),   # hidden test hooks
    (("solve", "-f", "x.cnf", "--run-chunk", "x"), "invalid value"),
    (("solve", "--share-devices"), "--input"),  # a flag without a value: parsing goes on to the required ones
])
def test_usage_errors(argv, needle):
    r = run(*argv)
    assert r.returncode == 2
    assert needle in r.stderr


def test_missing_file():
    r = run("solve", "-f", "/nonexistent/formula.cnf")
    assert r.returncode == 1 and "cannot read" in r.stderr


def test_malformed_formula(tmp_path):
    p = tmp_path / "bad.cnf"
    p.write_text("p cnf 3 1\n1 x 2 0\n")
    r = run("solve", "-f", str(p))
    assert r.returncode == 1 and "parse" in r.stderr


# ------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_solve_planted(tmp_path, dtype):
    p, clauses = planted(tmp_path)
    out = tmp_path / "out.txt"
    r = run("solve", "-f", str(p), "-s", "0.1", "-o", str(out), "--dtype", dtype)
    assert r.returncode == 0, r.stderr
    assert "Checking if solution vector satisfies formula: true" in r.stdout
    assert "Writing results to file..." in r.stdout
    assign = parse_render(out.read_text())
    assert sorted(assign) == list(range(1, 61))
    assert satisfies(assign, clauses)


@pytest.mark.gpu
def test_solve_adaptive_prints_assignment(golden_dir):
    r = run("solve", "-f", os.path.join(golden_dir, "small.cnf"))
    assert r.returncode == 0, r.stderr
    assert "satisfies formula: true" in r.stdout
    body = r.stdout.split("Variable assignments:\n", 1)[1]
    assert len(parse_render(body)) >= 1


@pytest.mark.gpu
def test_batch_unsat_reports_false(golden_dir):
    """aim-100-1_6-no-1 is unsatisfiable: every replica runs its -n steps, the last is reported."""
    r = run("batch", "-f", os.path.join(golden_dir, "hard.cnf"), "-n", "200", "-b", "4", "-s", "0.05")
    assert r.returncode == 0, r.stderr
    assert "\nChecking if solution vector satisfies formula: false" in r.stdout


@pytest.mark.gpu
def test_batch_and_inter_planted(tmp_path):
    p, clauses = planted(tmp_path, seed=9)
    for cmd in (("batch", "-n", "20000"), ("inter",)):
        out = tmp_path / f"{cmd[0]}.txt"
        r = run(cmd[0], "-f", str(p), *cmd[1:], "-b", "8", "-s", "0.1", "-o", str(out), "--seed", "5")
        assert r.returncode == 0, r.stderr
        assert "satisfies formula: true" in r.stdout, r.stdout
        assert satisfies(parse_render(out.read_text()), clauses)


@pytest.mark.gpu
def test_solve_preprocesses_then_rebuilds_eliminated_variables(golden_dir, tmp_path):
    """easy.cnf ("Edited to be Satisfiable"): preprocessing to ratio 7 leaves 267 clauses over 43
    variables (tests/golden/preprocess_golden.json); the trace restores the other 57."""
    out = tmp_path / "easy.txt"
    path = os.path.join(golden_dir, "easy.cnf")
    r = run("solve", "-f", path, "-s", "0.1", "-o", str(out))
    assert r.returncode == 0, r.stderr
    assert "Clauses: 267 | Vars: 43" in r.stdout
    assert "Mapping values..." in r.stdout and "satisfies formula: true" in r.stdout
    assign = parse_render(out.read_text())
    assert sorted(assign) == list(range(1, 101))
    with open(path) as fh:
        clauses = [ln for ln in fh.read().splitlines() if ln and ln[0] not in "cp%"]
    assert satisfies(assign, clauses)


@pytest.mark.gpu
def test_stoch_solves_easy(golden_dir, tmp_path):
    """main.rs:206-251: preprocessing, the discrete search from v = false, trace, check."""
    out = tmp_path / "stoch.txt"
    path = os.path.join(golden_dir, "easy.cnf")
    r = run("stoch", "-f", path, "-o", str(out), "--seed", "3")
    assert r.returncode == 0, r.stderr
    assert "Clauses: 267 | Vars: 43" in r.stdout and "satisfies formula: true" in r.stdout
    assign = parse_render(out.read_text())
    with open(path) as fh:
        clauses = [ln for ln in fh.read().splitlines() if ln and ln[0] not in "cp%"]
    assert satisfies(assign, clauses)


@pytest.mark.gpu
def test_stoch_bounded_on_unsat(golden_dir):
    r = run("stoch", "-f", os.path.join(golden_dir, "hard.cnf"), "-n", "300")
    assert r.returncode == 0, r.stderr
    assert "Checking if solution vector satisfies formula: false" in r.stdout
