"""The generated field asm blocks end without a wait-state guard (tools/gen_field_asm.py emit): their
SGPR outputs are dead temporaries, so no memory instruction may read an SGPR a block's VALU wrote
within the 5 wait states the gfx9 "VALU writes SGPR -> VMEM reads it" hazard needs.  This compiles
every kernel of the library for gfx950 (CPU only, hipcc) and follows each block exit."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_memory_read_of_block_written_sgprs():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asm_exit_check.py")], capture_output=True,
                       text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert r.stdout.strip().endswith("flags 0"), r.stdout[-500:]
