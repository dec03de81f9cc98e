"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

TEST INFRASTRUCTURE — runs only in the survey container, where
/root/reference exists and oracle/ref/build_ref.sh has built
oracle/_ref/c2d_refdrv (the reference's own Fortran + a serial driver).

For every case below it writes an input deck in the reference's format,
runs NSTEPS Monte-Carlo steps and stores, per step, the transport inputs the
reference computed (imcgen2d/volume_em/file_sp output) and the worker
tallies, census buffer and escape events it produced, as <case>.npz.
It also writes compton2d_amd/data/medium_inputm.npz: the per-cell tables
(kappa_tot, eps_tot, eps_th, f_nt, Pnt, emissivity) the reference computes
for the src_20121026/inputm.dat medium, used by compton2d_amd.synth to build
the benchmark's synthetic 32x32 workload.

usage: python tests/golden/make_golden.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import json
import shutil
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import refcase  # noqa: E402

# src_20121026/input.dat:113-116
PROD_SPLITS = dict(split1=1000, split2=1000, split3=300, spl3_trg=10)


def _c3_transport(nst: int) -> dict:
    """The C3 deck (compton2d_amd/synth.py C3_DECK) with T_const = 1: the
    transport inputs and tallies only (no FP_calc between steps)."""
    from compton2d_amd import synth
    d = synth.c3_refcase(nst=nst)
    d["T_const"] = 1
    for k in PROD_SPLITS:
        d.pop(k)
    return d


CASES = {
    # optically thicker SSC blob: collisions, split2/split3, census, escapes
    "ssc_tau": dict(case=dict(nz=2, nr=2, n_e=4.0e6, nst=2000), nsteps=3),
    # thin blob with an external-Compton seed spectrum on the lower boundary
    # (file_sample + r_surf_calc; disk/blackbody_20110929.in, hazard H9)
    "ec_lower": dict(case=dict(nz=2, nr=2, n_e=2.0e6, nst=1000, tbbl=-1.0), nsteps=3),
    # 3x4 grid, two angular bins
    "grid3x4": dict(case=dict(nz=3, nr=4, n_e=1.0e6, nst=1500, nmu=2), nsteps=2),
    # EC seed spectrum on the UPPER boundary (r_surf_calc's upper-ring loop,
    # src/imcsurf2d_para.f:362-420: wmu = -fibran(), zpre = z(nz), file_sample)
    "ec_upper": dict(case=dict(nz=2, nr=2, n_e=2.0e6, nst=1000, tbbu=-1.0), nsteps=3),
    # blackbody upper rings (tbbu > 0): planck (src/planck2d.f:1-141) on
    # upper-ring packets; src/imcgen2d.f:436-437 gives such rings no packets,
    # so the driver hands each 200 of weight erinu/200 (c2d_refdrv NFORCEU)
    "bb_upper": dict(case=dict(nz=2, nr=2, n_e=2.0e6, nst=1000, tbbu=[2.0e-3, 5.0e-2]),
                     nsteps=2, nforceu=200),
    # BASELINE C1: ONE zone, the inputm.dat medium, the EC
    # seed spectrum disk/blackbody_20110929.in on the lower ring (tbbl = -1,
    # the NaN-free file, H9); every flight ends at a system edge or census
    # (src/imctrk2d.f:276-360 with nz = nr = 1).  The EC window is kept open
    # (t0 = 0, t1 = 1e30) so the surface source runs every step.
    "c1_ec1x1": dict(case=dict(nz=1, nr=1, n_e=80.0, nst=20000, tbbl=-1.0), nsteps=3),
    # BASELINE C2: the 32x32 (r,z) grid of the inputm.dat medium, FP off: the
    # 1024-cell indexing, LDS-privatised tallies of 1024 cells (32 KB) and the
    # n_field of 1024 cells; nst = 2e5 so every cell is visited
    "c2_32x32": dict(case=dict(nz=32, nr=32, n_e=80.0, nst=200000), nsteps=2),
    # the 2012-11 snapshot's tracker (c2d_config.trk_variant = C2D_TRK_2012_11,
    # SURVEY.md §8 H1): src_20121113/imctrk2d.f + imcfield2d.f linked into
    # the driver (oracle/ref/build_ref.sh c2d_refdrv_2012) on ssc_tau's deck
    # (collisions, split3, census) and grid3x4's (12 cells, 2 angular bins)
    "ssc_tau_2012": dict(case=dict(nz=2, nr=2, n_e=4.0e6, nst=2000), nsteps=3, trk_variant=1),
    "grid3x4_2012": dict(case=dict(nz=3, nr=4, n_e=1.0e6, nst=1500, nmu=2), nsteps=2, trk_variant=1),
    # the production splits of the C3 deck (src_20121026/input.dat:113-116:
    # split1/2/3 = 1000/1000/300, spl3_trg = 10; SURVEY.md §8(d) "parity run").
    # C3's 30x9 grid and inputm.dat medium, FP off: the optically thin case,
    # where every source is 1000 probes (src/imctrk2d.f:105-138) -- on the GPU
    # 32 bundle restarts of up to 32 probes each (transport.hip bundle_begin)
    "prod_c3": dict(case=dict(PROD_SPLITS, **_c3_transport(nst=6000)), nsteps=2),
    # the same splits in a medium where split1 probes collide: n_e = 1e5
    # (tau_T ~ 5e-4, so 1000 probes see ~0.5 collisions per source and every
    # collision fans out to 1000 secondaries, src/imctrk2d.f:584-704; split3
    # fires on the gmax = 1e5 tail's >1e7 gains)
    "prod_dense": dict(case=dict(PROD_SPLITS, nz=2, nr=2, n_e=1.0e5, nst=60), nsteps=2),
}

# C3: the Mrk 421 SSC deck src_20121026/input.dat:1-130 +
# inputm.dat, transport AND Fokker-Planck, at reduced nst; see
# compton2d_amd/synth.py C3_DECK for the deviations (splits, rand_switch)
C3_CASE = "c3_mrk421"
C3_NST = 20000
C3_STEPS = 3

# Fokker-Planck cases (T_const=0): the reference's update/FP_calc after each
# transport step with ncycle > 0 (refdrv dumps fpin_/fpout_NNN.bin)
FP_CASES = {
    # constant Gaussian pick-up + turbulence heating (src_20121026/input.dat:97-105)
    "fp_pick": dict(case=dict(nz=2, nr=2, n_e=4.0e6, nst=400, T_const=0, pick_sw=1,
                              turb_lev=1.0e-2), nsteps=3),
    # shock injection (power law with moving cut-off) + coronal flare
    "fp_inj": dict(case=dict(nz=2, nr=2, n_e=4.0e6, nst=400, T_const=0, inj_switch=1, inj_dis=2,
                             g2var_switch=1, inj_t=0.0, inj_L=5e40, cf_sentinel=1,
                             flare_amp=10.0, t_flare=1.0e5, sigma_t=1.0e6, sigma_r=1.0e16,
                             sigma_z=1.0e16), nsteps=3),
    # C3's pair_switch = 1 (src_20121026/input.dat): pa_calc / trid_p / loop
    # 460 run with the MPI build's inert positrons (hazard H6)
    "fp_pair": dict(case=dict(nz=2, nr=2, n_e=4.0e6, nst=400, T_const=0, pick_sw=1,
                              turb_lev=1.0e-2, pair_switch=1), nsteps=3),
    # shock injection of a Gaussian (inj_dis = 1, src/update2d.f:1254-1258)
    # centred at the deck's inj_gg/inj_sigma, without the flare
    "fp_gauss": dict(case=dict(nz=2, nr=2, n_e=4.0e6, nst=400, T_const=0, inj_switch=1, inj_dis=1,
                               inj_t=0.0, inj_L=5e40, inj_gg=3.0e2, inj_sigma=3.0e1), nsteps=3),
}
FP_CONST_KEYS = ("cf_sentinel", "r_flare", "z_flare", "t_flare", "sigma_r", "sigma_z", "sigma_t",
                 "flare_amp", "r_esc", "r_acc", "inj_switch", "inj_dis", "g2var_switch", "pick_sw",
                 "inj_g1", "inj_g2", "inj_p", "inj_t", "inj_L", "pick_rate", "inj_gg", "inj_sigma",
                 "g_bulk")

TALLY_KEYS = ("edep", "prdep", "ecens", "npcen", "n_field", "E_IC", "nelectron", "fout", "edout",
              "erlki", "erlko", "erlku", "erlkl", "Ed_in", "census_d", "census_i", "events")
IN_KEYS = ("kappa_tot", "eps_tot", "eps_th", "f_nt", "Pnt", "n_e", "Eloss_th", "Eloss_tot",
           "zsurf", "ewsv", "nsv", "nsurfi", "nsurfo", "ewsurfi", "ewsurfo", "nsurfu", "nsurfl",
           "ewsurfu", "ewsurfl", "tbbi", "tbbo", "tbbu", "tbbl")


def run_case(name: str, spec: dict, out_dir: Path, work: Path, fp: bool = False) -> Path:
    d = work / name
    if d.exists():
        shutil.rmtree(d)
    refcase.write_input_deck(d, spec["case"])
    refcase.run_reference(d, spec["nsteps"], klag=1, nforceu=spec.get("nforceu", 0),
                          timeout=7200 if fp else 600, trk_variant=spec.get("trk_variant", 0))
    cfg = refcase.read_config(d)
    arrays = {}
    meta = {k: v for k, v in cfg.items() if not isinstance(v, np.ndarray)}
    meta["nsteps"] = spec["nsteps"]
    meta["trk_variant"] = spec.get("trk_variant", 0)
    meta["case"] = spec["case"]
    for k, v in cfg.items():
        if isinstance(v, np.ndarray):
            arrays["cfg_" + k] = v
    for n in range(spec["nsteps"]):
        si = refcase.read_step_in(d, n, cfg)
        so = refcase.read_step_out(d, n, cfg)
        if n == 0:
            arrays["E_ph"] = si["E_ph"]
        meta["step%d" % n] = dict(ncycle=si["ncycle"], ti=si["ti"], time=si["time"], dt=si["dt"],
                                  rseed_after=si["rseed_after"], nfile=so["nfile"])
        for k in IN_KEYS:
            arrays["in%d_%s" % (n, k)] = si[k]
        for k in TALLY_KEYS:
            arrays["out%d_%s" % (n, k)] = so[k]
        nf = so["nfile"]
        if nf >= 2:
            for k in ("E_file", "a1", "I_file", "F_file", "P_file"):
                arrays["out%d_%s" % (n, k)] = so[k][:nf]
    if fp:
        full = dict(refcase.BASE_CASE)
        full.update(spec["case"])
        meta["fp_const"] = {k: full[k] for k in FP_CONST_KEYS}
        steps = []
        for n in range(spec["nsteps"]):
            if not refcase.has_fp(d, n):
                continue
            fi, fo = refcase.read_fp_in(d, n, cfg), refcase.read_fp_out(d, n, cfg)
            steps.append(n)
            meta["fp%d" % n] = dict(ncycle=fi["ncycle"], time=fi["time"], dt=fi["dt"],
                                    **{k: fo[k] for k in ("E_tot_old", "E_tot_new", "hr_total",
                                                          "hr_st_total", "dT_max")})
            for k, v in fi.items():
                # the photon field/ecens FP_calc reads are this step's tallies (out%d_)
                if isinstance(v, np.ndarray) and k not in ("n_field", "ecens"):
                    arrays["fpin%d_%s" % (n, k)] = v
            for k, v in fo.items():
                if isinstance(v, np.ndarray):
                    arrays["fpout%d_%s" % (n, k)] = v
            assert np.array_equal(fi["n_field"], arrays["out%d_n_field" % n])
            assert np.array_equal(fi["ecens"], arrays["out%d_ecens" % n])
        meta["fp_steps"] = steps
        # the electron state passes unchanged between FP and transport
        # (fpin_n = in_n, in_n+1 = fpout_n): store each array once
        meta["alias"] = dedupe(arrays)
    arrays["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    path = out_dir / (name + ".npz")
    np.savez_compressed(path, **arrays)
    return path


def dedupe(arrays: dict) -> dict:
    """Drop arrays equal to one stored under an earlier key; returns
    {dropped key: kept key} (tests/golden_io.py resolves it)."""
    alias, seen = {}, {}
    for k in list(arrays):
        v = arrays[k]
        sig = (v.dtype.str, v.shape, hash(v.tobytes()))
        if sig in seen and np.array_equal(arrays[seen[sig]], v):
            alias[k] = seen[sig]
            del arrays[k]
        else:
            seen[sig] = k
    return alias


def c3_spec() -> dict:
    from compton2d_amd import synth
    return dict(case=synth.c3_refcase(nst=C3_NST), nsteps=C3_STEPS)


def run_fp_case(name: str, spec: dict, out_dir: Path, work: Path) -> Path:
    """FP inputs/outputs of the reference's update (update2d.f:7-327) per step."""
    d = work / name
    if d.exists():
        shutil.rmtree(d)
    refcase.write_input_deck(d, spec["case"])
    refcase.run_reference(d, spec["nsteps"], klag=1, timeout=3600)
    cfg = refcase.read_config(d)
    full = dict(refcase.BASE_CASE)
    full.update(spec["case"])
    meta = {k: v for k, v in cfg.items() if not isinstance(v, np.ndarray)}
    meta["case"] = spec["case"]
    meta["fp_const"] = {k: full[k] for k in FP_CONST_KEYS}
    arrays = {"cfg_" + k: v for k, v in cfg.items() if isinstance(v, np.ndarray)}
    arrays["E_ph"] = refcase.read_step_in(d, 0, cfg)["E_ph"]
    steps = []
    for n in range(spec["nsteps"]):
        if not refcase.has_fp(d, n):
            continue
        fi, fo = refcase.read_fp_in(d, n, cfg), refcase.read_fp_out(d, n, cfg)
        steps.append(n)
        meta["fp%d" % n] = dict(ncycle=fi["ncycle"], time=fi["time"], dt=fi["dt"],
                                **{k: fo[k] for k in ("E_tot_old", "E_tot_new", "hr_total",
                                                      "hr_st_total", "dT_max")})
        for k, v in fi.items():
            if isinstance(v, np.ndarray):
                arrays["fpin%d_%s" % (n, k)] = v
        for k, v in fo.items():
            if isinstance(v, np.ndarray):
                arrays["fpout%d_%s" % (n, k)] = v
    meta["fp_steps"] = steps
    arrays["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    path = out_dir / (name + ".npz")
    np.savez_compressed(path, **arrays)
    fic = out_dir / "fp_fic.npz"
    np.savez_compressed(fic, F_IC=refcase.read_fic(d),
                        source="F_IC(num_nt, nphfield) of the reference setup (icloss2d.f:1-64)")
    return path


def make_census_format(out_dir: Path, work: Path) -> Path:
    """The reference's own write_cens/read_cens (src/census2d.f) on a set of
    records covering the e14.7 edge cases; pins compton2d_amd/census_io.py."""
    import subprocess
    drv = ROOT / "oracle" / "_ref" / "c2d_censdrv"
    rng = np.random.default_rng(5)
    n = 200
    d = np.column_stack([rng.uniform(0, 7.5e15, n), rng.uniform(0, 1e16, n), rng.uniform(-1, 1, n),
                         rng.uniform(0, 6.3, n), 10 ** rng.uniform(30, 46, n),
                         10 ** rng.uniform(-7, 11, n)])
    d[0] = [0.0, -1.5e-5, -0.99999999, 6.2831853072, 9.999999951e45, 1.234567850e-7]
    d[1] = [1e-120, 5e120, 0.5, 1.0, 123456789.0, 0.099999995]
    i6 = np.column_stack([rng.integers(0, 129, n), rng.integers(0, 6, n), rng.integers(1, 33, n),
                          rng.integers(1, 100, n), rng.integers(1, 100, n),
                          rng.integers(0, 100000, n)]).astype(np.int32)
    w = work / "census"
    w.mkdir(parents=True, exist_ok=True)
    with open(w / "in.bin", "wb") as f:
        f.write(np.array([n], "<i4").tobytes())
        f.write(d.astype("<f8").tobytes())
        f.write(i6.astype("<i4").tobytes())
    subprocess.run([str(drv), "w", str(w / "in.bin"), str(w / "ref.txt")], check=True)
    subprocess.run([str(drv), "r", str(w / "ref.txt"), str(n), str(w / "back.bin")], check=True)
    back = np.fromfile(w / "back.bin", "<f8", count=6 * n).reshape(n, 6)
    iback = np.fromfile(w / "back.bin", "<i4", offset=48 * n).reshape(n, 6)
    text = (w / "ref.txt").read_bytes()
    path = out_dir / "census_fmt.npz"
    np.savez_compressed(path, d=d, i6=i6, text=np.frombuffer(text, np.uint8), read_d=back,
                        read_i=iback)
    return path


OBS_DECKS = {
    # the reference's own decks (postprocessing/mrk421_*.input)
    "sed_mrk421": ("pspt", "mrk421_sed.input"),
    "lc_mrk421": ("plcm", "mrk421_lc.input"),
    # decks that put most of the fixture's events into bins: several time and
    # energy bins, linear + log regions, three angular bins with defaulted
    # lower edges, overlapping bands, a time offset
    "sed_wide": ("pspt", "p001_evb.dat\n33\n1e16\nsed_w.dat\n12\n-4000\n2e4\n0.999\n1.0\n2\n"
                         "1e-4\n1e2\n24\n0\n1e2\n1e6\n8\n1\ny\n"),
    "lc_wide": ("plcm", "p001_evb.dat\n15\n1e17\nlc07_ev0.dat\n3\nlc07_ev0.dat\n0.97\n0.995\n"
                        "lc07_ev1.dat\n\n0.9995\nlc07_ev2.dat\n\n1.0001\n2e4\n4e4\n1.5e6\n4\n"
                        "1e-3\n1e1\n1\n0\n1\n1e3\n3\n0\n1e2\n1e6\n2\n1\n1e-4\n1e7\n1\n0\n"),
}


def make_observer(out_dir: Path, work: Path) -> Path:
    """The reference's post-processing tools (postprocessing/pspt.c, plcm.c,
    compiled by oracle/ref/build_ref.sh) run over the escape events the
    reference itself wrote in the golden transport cases, split over two
    event files (p001_evb.dat, p002_evb.dat) so the tools' file walk is
    exercised.  Stores events, decks and every output file."""
    import resource
    import subprocess
    from compton2d_amd import observer
    ev = []
    for case, steps in (("ssc_tau", (1, 2)), ("grid3x4", (1,)), ("ec_lower", (1, 2))):
        g = np.load(out_dir / ("%s.npz" % case))
        ev += [g["out%d_events" % s] for s in steps]
    ev = np.concatenate(ev)
    pp = Path("/root/reference/postprocessing")
    arrays = dict(events=ev, n_file1=np.array(len(ev) // 2))
    for name, (tool, deck) in OBS_DECKS.items():
        text = (pp / deck).read_text() if deck.endswith(".input") else deck
        d = work / "obs" / name
        if d.exists():
            shutil.rmtree(d)
        d.mkdir(parents=True)
        observer.write_events(d / "p001_evb.dat", ev[: len(ev) // 2])
        observer.write_events(d / "p002_evb.dat", ev[len(ev) // 2:])
        before = set(p.name for p in d.iterdir())

        def big_stack():
            resource.setrlimit(resource.RLIMIT_STACK, (resource.RLIM_INFINITY, resource.RLIM_INFINITY))
        subprocess.run([str(ROOT / "oracle" / "_ref" / tool)], input=text.encode(), cwd=d,
                       stdout=subprocess.DEVNULL, check=True, preexec_fn=big_stack)
        outs = sorted(p.name for p in d.iterdir() if p.name not in before)
        arrays["deck_" + name] = np.array(text)
        arrays["tool_" + name] = np.array(tool)
        arrays["files_" + name] = np.array(outs)
        for f in outs:
            arrays["out_%s__%s" % (name, f)] = np.array((d / f).read_text())
    path = out_dir / "obs.npz"
    np.savez_compressed(path, **arrays)
    return path


def vem_cells():
    """Cell states for the volume_em fixture: the inputm.dat medium, the
    reference's own f_nt of the FP fixtures (after FP steps), and draws that
    reach every branch (Theta < / > 0.2, the absorbed branch, nu <= nu_p)."""
    rng = np.random.default_rng(11)
    fnts = []
    for case in ("ssc_tau", "grid3x4"):
        g = np.load(HERE / ("%s.npz" % case))
        fnts += list(g["in0_f_nt"].reshape(-1, 200)[:2])
    for case in ("fp_pick", "fp_inj"):
        g = np.load(HERE / ("%s.npz" % case))
        for n in (1, 2):
            if "fpout%d_f_nt" % n in g.files:
                fnts += list(g["fpout%d_f_nt" % n].reshape(-1, 200)[:2])
    gnt = np.load(HERE / "ssc_tau.npz")["cfg_gnt"]
    cells = [  # T_keV, n_e, B, l_min
        (100.0, 80.0, 0.13, 3.75e15), (500.0, 4.0e6, 1.0, 1.0e15), (5.0, 1.0e3, 0.01, 5.0e15),
        (50.0, 1.0e10, 100.0, 1.0e13), (1000.0, 1.0e8, 10.0, 1.0e12), (102.0, 2.0e6, 0.13, 3.0e15),
        (300.0, 1.0e12, 1.0, 1.0e16),
    ]
    for _ in range(17):
        cells.append((10 ** rng.uniform(0.5, 3.0), 10 ** rng.uniform(0.0, 11.0),
                      10 ** rng.uniform(-2.0, 2.5), 10 ** rng.uniform(12.0, 16.0)))
    out = []
    for i, (T, ne, B, lm) in enumerate(cells):
        out.append(dict(T=T, ne=ne, B=B, l_min=lm, amxwl=0.0, gmin=1e2, gmax=1e5, p_nth=2.3,
                        f_pair=0.0, f_nt=np.asarray(fnts[i % len(fnts)], np.float64)))
    return gnt, out


def make_vem(out_dir: Path, work: Path) -> Path:
    """The reference's own volume_em (src/volume2d.f) on vem_cells(), through
    oracle/ref/c2d_vemdrv.f; pins oracle/c2d_vem_oracle.c."""
    import subprocess
    gnt, cells = vem_cells()
    w = work / "vem"
    w.mkdir(parents=True, exist_ok=True)
    with open(w / "in.bin", "wb") as f:
        f.write(np.array([len(cells)], "<i4").tobytes())
        f.write(np.asarray(gnt, "<f8").tobytes())
        for c in cells:
            f.write(np.array([c["T"], c["ne"], c["B"], c["l_min"], c["amxwl"], c["gmin"], c["gmax"],
                              c["p_nth"], c["f_pair"]], "<f8").tobytes())
            f.write(c["f_nt"].astype("<f8").tobytes())
    subprocess.run([str(ROOT / "oracle" / "_ref" / "c2d_vemdrv"), str(w / "in.bin"), str(w / "out.bin")],
                   check=True, stdout=subprocess.DEVNULL)
    raw = np.fromfile(w / "out.bin", "<f8")
    n = len(cells)
    E_ph = raw[:400]
    rec = raw[400:].reshape(n, 3 * 400 + 2)
    path = out_dir / "vem.npz"
    np.savez_compressed(
        path, gnt=gnt, E_ph=E_ph,
        state=np.array([[c["T"], c["ne"], c["B"], c["l_min"]] for c in cells]),
        f_nt=np.array([c["f_nt"] for c in cells]),
        kappa_tot=rec[:, :400], eps_tot=rec[:, 400:800], eps_th=rec[:, 800:1200],
        Eloss_cy=rec[:, 1200], Eloss_th=rec[:, 1201],
        source="reference volume_em (src/volume2d.f:10-394) via oracle/ref/c2d_vemdrv.f")
    return path


def make_medium(out_path: Path, work: Path) -> None:
    """Per-cell tables of the inputm.dat medium (n_e=80, B=0.13 G, p=2.3)."""
    d = work / "medium"
    if d.exists():
        shutil.rmtree(d)
    refcase.write_input_deck(d, dict(nz=1, nr=1, n_e=80.0, nst=200))
    refcase.run_reference(d, 1, klag=1)
    cfg = refcase.read_config(d)
    si = refcase.read_step_in(d, 0, cfg)
    vol = np.pi * cfg["r"][0] ** 2 * cfg["z"][0]
    np.savez_compressed(
        out_path, E_ph=si["E_ph"], gnt=cfg["gnt"], E_field=cfg["E_field"],
        kappa_tot=si["kappa_tot"][0, 0], eps_tot=si["eps_tot"][0, 0], eps_th=si["eps_th"][0, 0],
        f_nt=si["f_nt"][0, 0], Pnt=si["Pnt"][0, 0], n_e=si["n_e"][0, 0],
        emiss_per_vol_per_s=(si["Eloss_tot"][0, 0] / vol / si["dt"]),
        Eloss_th_frac=si["Eloss_th"][0, 0] / si["Eloss_tot"][0, 0],
        source="reference volume_em for src_20121026/inputm.dat (1x1 zone, R=7.5e15, Z=1e16)")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(HERE))
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    out = Path(args.out)
    with tempfile.TemporaryDirectory(prefix="c2d_golden_") as tmp:
        work = Path(tmp)
        for name, spec in CASES.items():
            if args.only and name != args.only:
                continue
            p = run_case(name, spec, out, work)
            print("wrote", p, p.stat().st_size, "bytes")
        for name, spec in FP_CASES.items():
            if args.only and name != args.only:
                continue
            p = run_fp_case(name, spec, out, work)
            print("wrote", p, p.stat().st_size, "bytes")
        if not args.only or args.only == C3_CASE:
            p = run_case(C3_CASE, c3_spec(), out, work, fp=True)
            print("wrote", p, p.stat().st_size, "bytes")
        if not args.only or args.only == "census_fmt":
            p = make_census_format(out, work)
            print("wrote", p, p.stat().st_size, "bytes")
        if not args.only or args.only == "vem":
            p = make_vem(out, work)
            print("wrote", p, p.stat().st_size, "bytes")
        if not args.only or args.only == "obs":
            p = make_observer(out, work)
            print("wrote", p, p.stat().st_size, "bytes")
        if not args.only:
            mp = ROOT / "compton2d_amd" / "data" / "medium_inputm.npz"
            mp.parent.mkdir(parents=True, exist_ok=True)
            make_medium(mp, work)
            print("wrote", mp, mp.stat().st_size, "bytes")


if __name__ == "__main__":
    main()
