"""The reference-side binding: a Fortran host holding the transport tables in
arrays with the reference's COMMON extents (jmax=kmax=99, n_vol=400,
num_nt=200) drives the engine through include/compton2d_mod.f90
(iso_c_binding) with the arrays passed in place via (c_loc, strides) —
the drop-in path for src/xec2d.f:167-176.  CPU: it compiles, links and fails
loudly without a GPU.  GPU: its tallies equal the Python host's on the same
golden inputs."""
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from compton2d_amd import abi
from golden_io import GoldenCase

ROOT = Path(__file__).resolve().parents[1]
FLANG = shutil.which("flang") or "/opt/rocm/lib/llvm/bin/flang"
BUILD = ROOT / "build" / "fortran"


def build_driver() -> Path:
    if not Path(FLANG).exists():
        pytest.skip("flang not available")
    BUILD.mkdir(parents=True, exist_ok=True)
    exe = BUILD / "fortran_driver"
    subprocess.run([FLANG, "-O2", "-J", str(BUILD), "-c", str(ROOT / "include" / "compton2d_mod.f90"),
                    "-o", str(BUILD / "compton2d_mod.o")], check=True)
    lib = ROOT / "compton2d_amd"
    subprocess.run([FLANG, "-O2", "-I", str(BUILD), str(ROOT / "examples" / "fortran_driver.f90"),
                    str(BUILD / "compton2d_mod.o"), "-L", str(lib), "-lcompton2d",
                    "-Wl,-rpath," + str(lib), "-o", str(exe)], check=True)
    return exe


def write_case(gc: GoldenCase, path: Path, nsteps: int, mode: int) -> None:
    g = gc.grid()
    with open(path, "wb") as f:
        hdr = [gc.nz, gc.nr, g.hu.size - 1, g.Elcmin.size, g.mu.size, nsteps, g.split1, g.split2,
               g.split3, g.spl3_trg, mode]
        f.write(np.array(hdr, "<i4").tobytes())
        f.write(np.array([g.rmin, g.zmin], "<f8").tobytes())
        for a in (g.z, g.r, g.E_ph, g.E_field, g.gnt, g.hu, g.Elcmin, g.Elcmax, g.mu):
            f.write(np.asarray(a, "<f8").tobytes())
        for n in range(nsteps):
            si = gc.step_inputs(n)
            f.write(np.array([si.ncycle], "<i4").tobytes())
            f.write(np.array([si.time, si.dt], "<f8").tobytes())
            for a in (si.kappa_tot, si.eps_tot, si.eps_th, si.f_nt, si.Pnt):   # [j][k][i]
                f.write(np.ascontiguousarray(a, "<f8").tobytes())
            for a in (si.n_e, si.Eloss_th, si.Eloss_tot, si.zsurf, si.ewsv):
                f.write(np.ascontiguousarray(a, "<f8").tobytes())
            f.write(np.ascontiguousarray(si.nsv, "<i4").tobytes())
            for a in (si.nsurfi, si.nsurfo, si.nsurfu, si.nsurfl):
                f.write(np.asarray(a, "<i4").tobytes())
            for a in (si.ewsurfi, si.ewsurfo, si.ewsurfu, si.ewsurfl, si.tbbi, si.tbbo,
                      si.tbbu, si.tbbl):
                f.write(np.asarray(a, "<f8").tobytes())


def test_fortran_binding_builds_and_fails_loudly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    exe = build_driver()
    gc = GoldenCase("ssc_tau")
    write_case(gc, tmp_path / "case.bin", 1, abi.COMTOT_EXACT)
    r = subprocess.run([str(exe), str(tmp_path / "case.bin"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True)
    assert r.returncode == 3
    assert "c2d_init failed: -2" in r.stdout and "ROCm" in r.stdout


@pytest.mark.gpu
def test_fortran_host_matches_python_host(tmp_path):
    from compton2d_amd.engine import Engine
    exe = build_driver()
    gc = GoldenCase("ssc_tau")
    nsteps = gc.nsteps
    write_case(gc, tmp_path / "case.bin", nsteps, abi.COMTOT_EXACT)
    r = subprocess.run([str(exe), str(tmp_path / "case.bin"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    # the RCCL all-reduce through the C-ABI (c2d_comm_init/c2d_allreduce_tallies)
    # ran every step and, with one rank, left the buffer bit for bit unchanged
    assert r.stdout.count("allreduce: bitwise identical (1 rank)") == nsteps, r.stdout
    assert "MISMATCH" not in r.stdout
    fort = np.fromfile(tmp_path / "out.bin", "<f8").reshape(nsteps, -1)
    eng = Engine(gc.grid(comtot_mode=abi.COMTOT_EXACT, census_capacity=1048576,
                         event_capacity=1048576, queue_capacity=262144))
    L = abi.tally_layout(gc.nz, gc.nr, gc.nmu)
    c0 = L["counters"][0]
    for n in range(nsteps):
        eng.transport_step(gc.step_inputs(n))
        py = eng.tallies_raw()
        np.testing.assert_array_equal(fort[n][c0:c0 + 9], py[c0:c0 + 9])
        np.testing.assert_allclose(fort[n], py, rtol=1e-11, atol=1e-13 * np.abs(py).max())
    eng.close()


# ---------------------------------------------------------------------------
# `call update` -> c2d_fp_step from the Fortran host (examples/fortran_fp_driver.f90)
# ---------------------------------------------------------------------------
FP_INT_KEYS = ("cf_sentinel", "inj_switch", "inj_dis", "g2var_switch", "pick_sw")
FP_DBL_KEYS = ("df_implicit", "df_T", "r_esc", "r_acc", "r_flare", "z_flare", "t_flare", "sigma_r",
               "sigma_z", "sigma_t", "flare_amp", "inj_g1", "inj_g2", "inj_p", "inj_t", "inj_L",
               "pick_rate", "inj_gg", "inj_sigma", "inj_v")
FP_ZONE_IN = ("tea", "tna", "n_e", "B_field", "Eloss_sy", "ecens", "ec_old", "turb_lev", "vol",
              "f_pair", "gmin", "gmax", "amxwl", "p_nth")
FP_ZONE_OUT = ("Te_new", "tea", "n_e", "gmin", "gmax", "amxwl", "p_nth")


def build_fp_driver() -> Path:
    build_driver()
    exe = BUILD / "fortran_fp_driver"
    lib = ROOT / "compton2d_amd"
    subprocess.run([FLANG, "-O2", "-I", str(BUILD), str(ROOT / "examples" / "fortran_fp_driver.f90"),
                    str(BUILD / "compton2d_mod.o"), "-L", str(lib), "-lcompton2d",
                    "-Wl,-rpath," + str(lib), "-o", str(exe)], check=True)
    return exe


def write_fp_case(fc, path: Path) -> None:
    g = fc.grid()
    k = fc.constants()
    with open(path, "wb") as f:
        f.write(np.array([fc.nz, fc.nr, g.hu.size - 1, g.Elcmin.size, g.mu.size, len(fc.steps)],
                         "<i4").tobytes())
        f.write(np.array([g.rmin, g.zmin], "<f8").tobytes())
        for a in (g.z, g.r, g.E_ph, g.E_field, g.gnt, g.hu, g.Elcmin, g.Elcmax, g.mu):
            f.write(np.asarray(a, "<f8").tobytes())
        f.write(np.array([getattr(k, n) for n in FP_INT_KEYS] + [0], "<i4").tobytes())
        f.write(np.array([getattr(k, n) for n in FP_DBL_KEYS] + [0.0, 0.0], "<f8").tobytes())
        f.write(np.asfortranarray(k.F_IC, "<f8").T.tobytes())     # F_IC(num_nt, nphfield)
        for n in fc.steps:
            fi = fc.fp_in(n)
            f.write(np.array([fi["ncycle"]], "<i4").tobytes())
            f.write(np.array([fi["time"], fi["dt"]], "<f8").tobytes())
            for key in FP_ZONE_IN:
                f.write(np.ascontiguousarray(fi[key], "<f8").tobytes())
            for key in ("f_nt", "Pnt", "n_field"):                      # [j][k][i]
                f.write(np.ascontiguousarray(fi[key], "<f8").tobytes())


def read_fp_out(path: Path, fc) -> list:
    raw = np.fromfile(path, "<f8")
    nz, nr, nt = fc.nz, fc.nr, abi.NUM_NT
    per = 5 + len(FP_ZONE_OUT) * nz * nr + 2 * nz * nr * nt
    out = []
    for s in range(len(fc.steps)):
        b = raw[s * per:(s + 1) * per]
        d = dict(zip(("E_tot_old", "E_tot_new", "hr_total", "hr_st_total", "dT_max"), b[:5]))
        o = 5
        for key in FP_ZONE_OUT:
            d[key] = b[o:o + nz * nr].reshape(nz, nr)
            o += nz * nr
        for key in ("f_nt", "Pnt"):
            d[key] = b[o:o + nz * nr * nt].reshape(nz, nr, nt)
            o += nz * nr * nt
        out.append(d)
    return out


def test_fortran_fp_binding_builds_and_fails_loudly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    from golden_io import FpGoldenCase
    exe = build_fp_driver()
    fc = FpGoldenCase("fp_pick")
    write_fp_case(fc, tmp_path / "fp.bin")
    r = subprocess.run([str(exe), str(tmp_path / "fp.bin"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True)
    assert r.returncode == 3
    assert "c2d_init failed: -2" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name", ("fp_pick", "fp_inj"))
def test_fortran_fp_host_matches_python_host(tmp_path, name):
    """COMMON-extent arrays updated in place by c2d_fp_step equal the Python
    host's result, which equals the reference's FP_calc (tests/test_gpu_fp.py)."""
    from golden_io import FpGoldenCase
    from compton2d_amd.engine import Engine
    exe = build_fp_driver()
    fc = FpGoldenCase(name)
    write_fp_case(fc, tmp_path / "fp.bin")
    r = subprocess.run([str(exe), str(tmp_path / "fp.bin"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    fort = read_fp_out(tmp_path / "out.bin", fc)
    eng = Engine(fc.grid(device=0))
    eng.fp_set_config(fc.constants())
    for s, n in enumerate(fc.steps):
        fi = fc.fp_in(n)
        py = eng.fp_step(fi["ncycle"], fi["time"], fi["dt"], fi, fi)
        for key in FP_ZONE_OUT + ("f_nt", "Pnt"):
            np.testing.assert_array_equal(fort[s][key], py[key], err_msg=key)
        for key in ("E_tot_old", "E_tot_new", "hr_total", "hr_st_total", "dT_max"):
            assert fort[s][key] == py[key], key
        np.testing.assert_array_equal(py["Te_new"], fc.fp_out(n)["Te_new"])
    eng.close()
