#!/usr/bin/env python3
"""How fast is the CPU baseline's C port against the reference's own Fortran?

TEST INFRASTRUCTURE - runs only in the survey container (the reference's
Fortran, built by oracle/ref/build_ref.sh into oracle/_ref/, does not travel).

bench.py's cpu_baseline times the C oracle in its reference mode (per-copy
split1 probes, the lagged-Fibonacci zone streams with the per-census-packet
reseed of src/imcfield2d.f:115-116 / src/rand.f:99-122,260-316, exact comtot,
glibc libm).  That port is bit-exact to the Fortran (tests/test_oracle_golden.py)
but not the same code, so its speed is not the reference's speed.  This tool
runs the SAME transport work through both, one process each, on this
container's cores:

  1. the reference's serial driver oracle/_ref/c2d_refdrv on the C3 deck
     (synth.c3_refcase, T_const = 1 so no FP_calc runs between steps) for
     --steps steps at --nst; it times its own census (field_calc), volume
     (vol_calc) and surface legs per step (transport_times.txt);
  2. the C oracle (glibc build, fib streams, h4_stale) on the inputs the
     driver dumped for each step (in_NNN.bin), its census carried from its
     own previous step -- the identical histories: every tally and the
     census are compared bit for bit with the driver's out_NNN.bin.

Both do the same packet-steps (the oracle counts them, C2D_CNT_STEPS).  The
Fortran writes one e14.7 text line per escape (imcleak2d.f:171) inside its
timed legs; the port keeps events in memory.

usage: python tools/fortran_vs_port.py [--nst 20000] [--steps 4] [--out FILE.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle_lib as OL  # noqa: E402
import refcase  # noqa: E402
from compton2d_amd import abi, synth  # noqa: E402

EXACT = ("edep", "prdep", "ecens", "npcen", "n_field", "edout")


def grid_of(cfg: dict, E_ph: np.ndarray) -> abi.GridConfig:
    return abi.GridConfig(
        nz=cfg["nz"], nr=cfg["nr"], rmin=cfg["rmin"], zmin=cfg["zmin"], z=cfg["z"], r=cfg["r"],
        E_ph=E_ph, E_field=cfg["E_field"], gnt=cfg["gnt"], hu=cfg["hu"], Elcmin=cfg["Elcmin"],
        Elcmax=cfg["Elcmax"], mu=cfg["mu"], split1=cfg["split1"], split2=cfg["split2"],
        split3=cfg["split3"], spl3_trg=cfg["spl3_trg"], spec_switch=cfg["spec_switch"],
        cr_sent=cfg["cr_sent"], pair_switch=cfg["pair_switch"])


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nst", type=int, default=20000)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    deck = synth.c3_refcase(nst=args.nst)
    deck["T_const"] = 1
    with tempfile.TemporaryDirectory(prefix="c2d_fvp_") as tmp:
        d = Path(tmp) / "c3"
        refcase.write_input_deck(d, deck)
        t0 = time.perf_counter()
        refcase.run_reference(d, args.steps, klag=1, timeout=7200)
        t_drv = time.perf_counter() - t0
        tt = np.loadtxt(d / "transport_times.txt", ndmin=2)
        cfg = refcase.read_config(d)
        ins = [refcase.read_step_in(d, n, cfg) for n in range(args.steps)]
        outs = [refcase.read_step_out(d, n, cfg) for n in range(args.steps)]
        o = OL.Oracle(grid_of(cfg, ins[0]["E_ph"]), OL.RNG_FIB, "ref", rand_switch=cfg["rand_switch"],
                      rseed=cfg["rseed"], h4_stale=1)
        rows = []
        for n in range(args.steps):
            si = abi.StepInputs(ncycle=ins[n]["ncycle"], time=ins[n]["time"], dt=ins[n]["dt"], spectra=[],
                                **{k: ins[n][k] for k in refcase_in_keys()})
            t0 = time.perf_counter()
            rc = o.step(si)
            t_port = time.perf_counter() - t0
            assert rc == 0
            t = o.split()
            for k in EXACT:
                ref = outs[n][k].astype(np.float64)
                got = np.asarray(t[k], np.float64)[:ref.size].reshape(ref.shape)
                assert np.array_equal(got, ref), (n, k)
            d6, _, _ = o.census()
            assert np.array_equal(d6, outs[n]["census_d"]), n
            steps = float(t["counters"][abi.CNT_STEPS])
            t_f = float(tt[n, 1] + tt[n, 2] + tt[n, 3])
            rows.append(dict(step=n, packet_steps=steps, census_in=int(len(outs[n - 1]["census_d"])) if n else 0,
                             fortran_s=t_f, fortran_census_s=float(tt[n, 1]), fortran_volume_s=float(tt[n, 2]),
                             fortran_surface_s=float(tt[n, 3]), port_s=t_port,
                             port_speed_vs_fortran=t_f / t_port if t_port > 0 else None))
            print("step %d: %.4g packet-steps  Fortran %.3f s (census %.3f, volume %.3f)  port %.3f s  ratio %.2f"
                  % (n, steps, t_f, tt[n, 1], tt[n, 2], t_port, t_f / t_port), flush=True)
        o.close()
        ps = sum(r["packet_steps"] for r in rows)
        tf = sum(r["fortran_s"] for r in rows)
        tp = sum(r["port_s"] for r in rows)
        res = dict(deck="C3 (synth.c3_refcase, T_const=1)", nst=args.nst, steps=args.steps,
                   packet_steps=ps, fortran_s=tf, port_s=tp,
                   fortran_packet_steps_per_s=ps / tf, port_packet_steps_per_s=ps / tp,
                   port_speed_vs_fortran=tf / tp, driver_wall_s=t_drv, bitwise=True, per_step=rows,
                   method="one process each on this container's cores; Fortran = oracle/_ref/c2d_refdrv "
                          "(reference objects, flang -O2), transport legs timed with MPI_WTIME; port = "
                          "oracle/c2d_oracle.c glibc build in reference (fib) mode, c2o_step timed")
        print(json.dumps({k: v for k, v in res.items() if k != "per_step"}))
        if args.out:
            Path(args.out).write_text(json.dumps(res, indent=1) + "\n")


def refcase_in_keys():
    return ("kappa_tot", "eps_tot", "eps_th", "f_nt", "Pnt", "n_e", "Eloss_th", "Eloss_tot", "zsurf",
            "ewsv", "nsv", "nsurfi", "nsurfo", "ewsurfi", "ewsurfo", "nsurfu", "nsurfl", "ewsurfu",
            "ewsurfl", "tbbi", "tbbo", "tbbu", "tbbl")


if __name__ == "__main__":
    main()
