"""The C-ABI library: it loads without a GPU, exports every function that
include/compton2d.h declares, and its struct layouts match the ctypes mirror."""
import ctypes as C
import re
import subprocess
import tempfile
from pathlib import Path

import pytest

from compton2d_amd import abi, engine

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "compton2d.h"


def declared_functions():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(c2d_\w+)\s*\(", txt, flags=re.M))
                  - {"c2d_tally_layout_for"})


def test_library_loads_and_exports_every_declared_symbol():
    lib = engine.load_library()
    assert lib.c2d_version().startswith(b"compton2d_amd")
    out = subprocess.run(["nm", "-D", "--defined-only", str(engine.LIB_PATH)],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (c2d_\w+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    assert len(declared_functions()) >= 20


def test_struct_layouts_match_header():
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "compton2d.h"
#define P(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("c2d_config %zu\nc2d_step_in %zu\nc2d_tally_layout %zu\nc2d_fp_in %zu\nc2d_spectrum %zu\n",
         sizeof(c2d_config), sizeof(c2d_step_in), sizeof(c2d_tally_layout), sizeof(c2d_fp_in),
         sizeof(c2d_spectrum));
  printf("c2d_fp_config %zu\nc2d_fp_step_in %zu\nc2d_fp_step_out %zu\n", sizeof(c2d_fp_config),
         sizeof(c2d_fp_step_in), sizeof(c2d_fp_step_out));
  P(c2d_fp_config, inj_v) P(c2d_fp_config, F_IC_s_ph) P(c2d_fp_config, pick_sw)
  P(c2d_fp_step_in, n_field) P(c2d_fp_step_in, ecens) P(c2d_fp_step_in, dt)
  P(c2d_fp_step_out, zone_diag) P(c2d_fp_step_out, dT_max) P(c2d_fp_step_out, p_nth)
  P(c2d_config, seed) P(c2d_config, rank) P(c2d_config, queue_capacity) P(c2d_config, mu)
  P(c2d_config, census_inplace) P(c2d_config, trk_variant)
  P(c2d_step_in, kappa_tot) P(c2d_step_in, nsv) P(c2d_step_in, tbbl) P(c2d_step_in, spectra)
  P(c2d_step_in, n_spectra) P(c2d_step_in, dt) P(c2d_step_in, device_tables)
  printf("c2d_obs_bins %zu\nc2d_vem_in %zu\nc2d_vem_out %zu\n", sizeof(c2d_obs_bins),
         sizeof(c2d_vem_in), sizeof(c2d_vem_out));
  P(c2d_vem_in, ep_switch) P(c2d_vem_in, f_nt) P(c2d_vem_out, E_ph) P(c2d_vem_out, Eloss_tot)
  P(c2d_obs_bins, t_offset) P(c2d_obs_bins, t1) P(c2d_obs_bins, n_mu) P(c2d_obs_bins, E1)
  return 0;
}
'''
    with tempfile.TemporaryDirectory() as d:
        c = Path(d) / "l.c"
        c.write_text(src)
        exe = Path(d) / "l"
        subprocess.run(["gcc", "-I", str(ROOT / "include"), str(c), "-o", str(exe)], check=True)
        out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    got = dict(line.rsplit(" ", 1) for line in out.strip().splitlines())
    assert int(got["c2d_config"]) == C.sizeof(abi.Config)
    assert int(got["c2d_step_in"]) == C.sizeof(abi.StepIn)
    assert int(got["c2d_tally_layout"]) == C.sizeof(abi.TallyLayout)
    assert int(got["c2d_fp_in"]) == C.sizeof(abi.FpIn)
    assert int(got["c2d_spectrum"]) == C.sizeof(abi.Spectrum)
    assert int(got["c2d_fp_config"]) == C.sizeof(abi.FpConfig)
    assert int(got["c2d_fp_step_in"]) == C.sizeof(abi.FpStepIn)
    assert int(got["c2d_fp_step_out"]) == C.sizeof(abi.FpStepOut)
    assert int(got["c2d_obs_bins"]) == C.sizeof(abi.ObsBins)
    assert int(got["c2d_vem_in"]) == C.sizeof(abi.VemIn)
    assert int(got["c2d_vem_out"]) == C.sizeof(abi.VemOut)
    classes = {"c2d_config": abi.Config, "c2d_step_in": abi.StepIn, "c2d_fp_config": abi.FpConfig,
               "c2d_fp_step_in": abi.FpStepIn, "c2d_fp_step_out": abi.FpStepOut,
               "c2d_obs_bins": abi.ObsBins, "c2d_vem_in": abi.VemIn, "c2d_vem_out": abi.VemOut}
    for key, val in got.items():
        if "." in key:
            t, f = key.split(".")
            cls = classes[t]
            assert getattr(cls, f).offset == int(val), key


def test_tally_layout_python_matches_c():
    import oracle_lib as OL
    from golden_io import GoldenCase
    g = GoldenCase("grid3x4")
    o = OL.Oracle(g.grid(), OL.RNG_LINEAGE, "det")
    assert o.tallies().size == abi.tally_layout(3, 4, 2)["total"][0]
    o.close()


def test_init_fails_loudly_without_gpu():
    """No silent CPU fallback: without a device c2d_init reports a HIP error."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from golden_io import GoldenCase
    with pytest.raises(engine.C2DError) as e:
        engine.Engine(GoldenCase("ssc_tau").grid())
    assert "C2D_E_HIP" in str(e.value)


def test_init_rejects_event_capacity_below_shard_count():
    """The escape-event buffer is C2D_EV_SHARDS (32) equal shards: a smaller
    capacity would give every shard 0 slots: C2D_E_ARG before any
    device call."""
    from golden_io import GoldenCase
    g = GoldenCase("ssc_tau").grid(event_capacity=31)
    with pytest.raises(engine.C2DError) as e:
        engine.Engine(g)
    assert "C2D_E_ARG" in str(e.value)


def test_init_rejects_an_unknown_tracker_variant():
    """c2d_config.trk_variant is C2D_TRK_SRC (0) or C2D_TRK_2012_11 (1)."""
    from golden_io import GoldenCase
    g = GoldenCase("ssc_tau").grid(trk_variant=2)
    with pytest.raises(engine.C2DError) as e:
        engine.Engine(g)
    assert "C2D_E_ARG" in str(e.value)
