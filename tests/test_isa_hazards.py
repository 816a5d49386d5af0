"""Static ISA check of the asm LDS-read discipline (CPU; hipcc cross-compiles gfx950).

The MLP kernels read LDS through inline asm and publish each result with their own
counted `s_waitcnt lgkmcnt` (a compiler-visible LDS load would make hipcc drain every
in-flight LDS-DMA first).  The compiler then treats those registers as written at once,
so any instruction it places between such a read and its covering wait that touches
the register works on the old contents -- the fused backward had exactly that (a copy
on a branch edge).  tools/lds_hazard.py scans the gfx950 assembly of csrc/mlp.hip
(default model instances, -DNR_MLP_DEV) for it; every kernel must be clean."""

import importlib.util
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _checker():
    spec = importlib.util.spec_from_file_location("lds_hazard", ROOT / "tools" / "lds_hazard.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_checker_flags_a_copy_before_the_wait():
    chk = _checker()
    lines = ["\t;;#ASMSTART", "\tds_read_b64_tr_b16 v[86:87], v87 offset:0x2000", "\t;;#ASMEND",
             "\tv_mov_b64_e32 v[186:187], v[86:87]", "\ts_waitcnt lgkmcnt(0)",
             "\tv_mfma_f32_32x32x16_bf16 a[0:15], v[86:89], v[90:93], a[0:15]"]
    assert chk.scan(list(enumerate(lines, 1)), "synthetic") == 1
    ok = lines[:3] + ["\ts_waitcnt lgkmcnt(0)", "\tv_mov_b64_e32 v[186:187], v[86:87]"]
    assert chk.scan(list(enumerate(ok, 1)), "synthetic") == 0


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
def test_mlp_kernels_have_no_asm_lds_read_hazards(tmp_path):
    src = ROOT / "robust-nerf_amd" / "csrc" / "mlp.hip"
    out = tmp_path / "mlp_dev.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-ffp-contract=off",
                    "-DNR_MLP_DEV", f"-I{ROOT / 'include'}", f"-I{src.parent}", "--cuda-device-only", "-S", str(src),
                    "-o", str(out)], check=True, capture_output=True, timeout=600)
    chk = _checker()
    text = out.read_text().split("\n")
    import re
    starts = [i for i, x in enumerate(text) if re.match(r"^_Z\w+:", x)]
    assert starts, "no kernels in the assembly"
    total = 0
    for si, s in enumerate(starts):
        e = starts[si + 1] if si + 1 < len(starts) else len(text)
        total += chk.scan([(i + 1, text[i]) for i in range(s, e)], text[s].split(":")[0][:60])
    assert total == 0, f"{total} asm-read register hazard(s) in csrc/mlp.hip (see tools/lds_hazard.py)"
