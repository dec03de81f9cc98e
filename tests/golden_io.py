"""Load the golden fixtures of tests/golden/ (made by tests/golden/make_golden.py
from the reference itself) into compton2d_amd.abi structures — TEST INFRASTRUCTURE."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from compton2d_amd import abi

GOLDEN = Path(__file__).resolve().parent / "golden"
CASES = ("ssc_tau", "ec_lower", "grid3x4", "ec_upper", "bb_upper", "c3_mrk421", "c1_ec1x1",
         "c2_32x32", "ssc_tau_2012", "grid3x4_2012", "prod_c3", "prod_dense")
IN_KEYS = ("kappa_tot", "eps_tot", "eps_th", "f_nt", "Pnt", "n_e", "Eloss_th", "Eloss_tot",
           "zsurf", "ewsv", "nsv", "nsurfi", "nsurfo", "ewsurfi", "ewsurfo", "nsurfu", "nsurfl",
           "ewsurfu", "ewsurfl", "tbbi", "tbbo", "tbbu", "tbbl")


def _load(name: str):
    """(arrays, meta) of a fixture, with de-duplicated arrays restored
    (make_golden.dedupe: meta['alias'] maps a dropped key to its equal)."""
    z = np.load(GOLDEN / (name + ".npz"), allow_pickle=False)
    a = {k: z[k] for k in z.files}
    meta = json.loads(bytes(a.pop("meta_json")).decode())
    for k, src in meta.get("alias", {}).items():
        a[k] = a[src]
    return a, meta


class GoldenCase:
    def __init__(self, name: str):
        self.name = name
        self.a, self.meta = _load(name)
        self.nsteps = self.meta["nsteps"]
        self.nz, self.nr, self.nmu = self.meta["nz"], self.meta["nr"], self.meta["nmu"]

    def grid(self, **over) -> abi.GridConfig:
        m, a = self.meta, self.a
        g = abi.GridConfig(
            nz=m["nz"], nr=m["nr"], rmin=m["rmin"], zmin=m["zmin"], z=a["cfg_z"], r=a["cfg_r"],
            E_ph=a["E_ph"], E_field=a["cfg_E_field"], gnt=a["cfg_gnt"], hu=a["cfg_hu"],
            Elcmin=a["cfg_Elcmin"], Elcmax=a["cfg_Elcmax"], mu=a["cfg_mu"], split1=m["split1"],
            split2=m["split2"], split3=m["split3"], spl3_trg=m["spl3_trg"],
            spec_switch=m["spec_switch"], cr_sent=m["cr_sent"], pair_switch=m["pair_switch"],
            trk_variant=m.get("trk_variant", 0))
        for k, v in over.items():
            setattr(g, k, v)
        return g

    def step_inputs(self, n: int) -> abi.StepInputs:
        st = self.meta["step%d" % n]
        spectra = []
        if st["nfile"] >= 2 and ("out%d_E_file" % n) in self.a:
            spectra.append(abi.SpectrumTable(*(self.a["out%d_%s" % (n, k)] for k in
                                               ("E_file", "a1", "I_file", "F_file", "P_file"))))
        return abi.StepInputs(ncycle=st["ncycle"], time=st["time"], dt=st["dt"], spectra=spectra,
                              **{k: self.a["in%d_%s" % (n, k)] for k in IN_KEYS})

    def out(self, n: int, key: str) -> np.ndarray:
        return self.a["out%d_%s" % (n, key)]


FP_CASES = ("fp_pick", "fp_inj", "fp_pair", "fp_gauss")


def fp_fic() -> np.ndarray:
    """F_IC(num_nt, nphfield) of the reference setup, [NUM_NT, NPHFIELD]."""
    return np.load(GOLDEN / "fp_fic.npz", allow_pickle=False)["F_IC"]


class FpGoldenCase:
    """Inputs and outputs of the reference's `update` (FP_calc for every zone)
    per MC step, dumped by oracle/ref/c2d_refdrv.f (tests/golden/make_golden.py)."""

    def __init__(self, name: str):
        self.name = name
        self.a, self.meta = _load(name)
        self.steps = list(self.meta["fp_steps"])
        self.nz, self.nr = self.meta["nz"], self.meta["nr"]

    def grid(self, **over) -> abi.GridConfig:
        m, a = self.meta, self.a
        g = abi.GridConfig(
            nz=m["nz"], nr=m["nr"], rmin=m["rmin"], zmin=m["zmin"], z=a["cfg_z"], r=a["cfg_r"],
            E_ph=a["E_ph"], E_field=a["cfg_E_field"], gnt=a["cfg_gnt"], hu=a["cfg_hu"],
            Elcmin=a["cfg_Elcmin"], Elcmax=a["cfg_Elcmax"], mu=a["cfg_mu"])
        for k, v in over.items():
            setattr(g, k, v)
        return g

    def constants(self) -> abi.FpConstants:
        return abi.FpConstants(F_IC=fp_fic(), pair_switch=int(self.meta.get("pair_switch", 0)),
                               **self.meta["fp_const"])

    def fp_in(self, n: int) -> dict:
        d = {k[len("fpin%d_" % n):]: v for k, v in self.a.items() if k.startswith("fpin%d_" % n)}
        d.update({k: self.meta["fp%d" % n][k] for k in ("ncycle", "time", "dt")})
        return d

    def fp_out(self, n: int) -> dict:
        d = {k[len("fpout%d_" % n):]: v for k, v in self.a.items() if k.startswith("fpout%d_" % n)}
        d.update({k: self.meta["fp%d" % n][k] for k in ("E_tot_old", "E_tot_new", "hr_total",
                                                       "hr_st_total", "dT_max")})
        return d


class CoupledGoldenCase(GoldenCase):
    """Transport AND Fokker-Planck steps of one reference run (c3_mrk421:
    the C3 deck, tests/golden/make_golden.py): per step the transport inputs
    and tallies (GoldenCase) and, for ncycle > 0, the FP_calc inputs/outputs
    whose photon field / ecens are that step's tallies."""

    def __init__(self, name: str):
        super().__init__(name)
        self.fp_steps = list(self.meta["fp_steps"])

    def constants(self) -> abi.FpConstants:
        return abi.FpConstants(F_IC=fp_fic(), pair_switch=int(self.meta.get("pair_switch", 0)),
                               **self.meta["fp_const"])

    def fp_in(self, n: int) -> dict:
        d = {k[len("fpin%d_" % n):]: v for k, v in self.a.items() if k.startswith("fpin%d_" % n)}
        d["n_field"] = self.out(n, "n_field")
        d["ecens"] = self.out(n, "ecens")
        d.update({k: self.meta["fp%d" % n][k] for k in ("ncycle", "time", "dt")})
        return d

    def fp_out(self, n: int) -> dict:
        d = {k[len("fpout%d_" % n):]: v for k, v in self.a.items() if k.startswith("fpout%d_" % n)}
        d.update({k: self.meta["fp%d" % n][k] for k in ("E_tot_old", "E_tot_new", "hr_total",
                                                       "hr_st_total", "dT_max")})
        return d
