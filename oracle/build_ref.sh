#!/usr/bin/env bash
# build_ref.sh — TEST INFRASTRUCTURE ONLY.
#
# Compiles the reference's own host C++ sources, where they lie under
# /root/reference, into oracle/_ref/libbpref.so (git-ignored; travels to the
# GPU box as a binary, the sources never do).  Recipe = SURVEY Appendix A:
#   * g++ -x c++ on curve25519_ops.cu, bulletproof_vectors.cu,
#     bulletproof_challenge.cu, bulletproof_range_proof.cu (+ -include
#     cuda_bulletproof.h, the declaration missing at bulletproof_range_proof.cu:724),
#     complete_bulletproof_test.cu (-Dmain=ref_test_main, for its base-point generator);
#   * cuda_range_proof_verify.cu exists only inside the notebook (cell at
#     cudabulletproofoptimized.ipynb:6529); it is extracted to a private temp
#     dir for the compile and deleted afterwards — nothing lands in the repo;
#   * oracle/ref/ref_harness.cc (ours): host emulation of the GPU symbols over the
#     reference's device primitives, deterministic RAND_bytes, flat ctypes API.
# Links OpenSSL libcrypto (system package) as the reference does.
set -euo pipefail
REF=${REF:-/root/reference}
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
if [ ! -d "$REF" ]; then
    echo "build_ref.sh: $REF not present (expected on the GPU box); keeping prebuilt $OUT" >&2
    exit 0
fi
mkdir -p "$OUT"
TMP="$(mktemp -d)"
trap 'rm -rf "$TMP"' EXIT
python3 - "$REF/cudabulletproofoptimized.ipynb" "$TMP" <<'EOF'
import json, sys
nb = json.load(open(sys.argv[1]))
for c in nb["cells"]:
    src = "".join(c["source"])
    if src.startswith("%%writefile cuda_range_proof_verify.cu"):
        open(sys.argv[2] + "/cuda_range_proof_verify.cu", "w").write(src.split("\n", 1)[1])
        break
else:
    sys.exit("notebook cell for cuda_range_proof_verify.cu not found")
EOF
F="-O2 -w -x c++ -fPIC -I$REF"
cd "$TMP"
g++ $F -c "$REF/curve25519_ops.cu" -o curve25519_ops.o
g++ $F -c "$REF/bulletproof_vectors.cu" -o bulletproof_vectors.o
g++ $F -c "$REF/bulletproof_challenge.cu" -o bulletproof_challenge.o
g++ $F -include cuda_bulletproof.h -c "$REF/bulletproof_range_proof.cu" -o bulletproof_range_proof.o
g++ $F -D__device__= -c "$TMP/cuda_range_proof_verify.cu" -o cuda_range_proof_verify.o
g++ $F -Dmain=ref_test_main -c "$REF/complete_bulletproof_test.cu" -o complete_bulletproof_test.o
g++ -O2 -w -fPIC -I"$REF" -D__device__= -c "$HERE/ref/ref_harness.cc" -o ref_harness.o
g++ -shared -Wl,-Bsymbolic -o "$OUT/libbpref.so" *.o -lcrypto
echo "built $OUT/libbpref.so"

# The reference's own test driver (complete_bulletproof_test.cu, main() unchanged), three ways.
# Built with clang's -ftrivial-auto-var-init=pattern so that the driver's own undefined behaviour
# at its end — complete_bulletproof_test.cu:305 range_proof_free(&large_proof) frees the
# never-initialised ip_proof of the refused out-of-range proof (generate_range_proof returns early
# at bulletproof_range_proof.cu:1176-1187 before range_proof_init) — ends the same way on every run:
# free(0xaaaaaaaaaaaaaaaa) -> SIGSEGV, after all of its output.  (g++ builds leave stack garbage
# there: the run exits 0, SIGSEGVs or aborts in glibc depending on what the stack held.)
#   complete_bulletproof_test_cpu   GPU symbols host-emulated by ref_harness.cc (the CPU twin)
#   complete_bulletproof_test_asan  the same under AddressSanitizer + UBSan (tests/test_dropin.py
#                                   asserts the report: field_vector_free <- inner_product_proof_free
#                                   <- main at complete_bulletproof_test.cu:305, no UBSan finding)
#   complete_bulletproof_test_hip   linked against OUR libcudabulletproof_hip.so (the drop-in)
CXX=${CXX_PATTERN:-/opt/rocm/llvm/bin/clang++}
P="-O2 -w -x c++ -fPIC -I$REF -ftrivial-auto-var-init=pattern"
A="-O1 -g -w -x c++ -fPIC -I$REF -ftrivial-auto-var-init=pattern -fsanitize=address,undefined -fno-omit-frame-pointer"
for v in p a; do
    FL=$P; [ $v = a ] && FL=$A
    for f in curve25519_ops bulletproof_vectors bulletproof_challenge complete_bulletproof_test; do
        $CXX $FL -c "$REF/$f.cu" -o "${v}_$f.o"
    done
    $CXX $FL -include cuda_bulletproof.h -c "$REF/bulletproof_range_proof.cu" -o "${v}_bulletproof_range_proof.o"
    $CXX $FL -D__device__= -c "$TMP/cuda_range_proof_verify.cu" -o "${v}_crv.o"
    $CXX ${FL/-x c++/} -D__device__= -c "$HERE/ref/ref_harness.cc" -o "${v}_harness.o"
done
DRV="curve25519_ops bulletproof_vectors bulletproof_challenge bulletproof_range_proof complete_bulletproof_test"
$CXX -o "$OUT/complete_bulletproof_test_cpu" $(for f in $DRV crv harness; do echo p_$f.o; done) -lcrypto
$CXX -fsanitize=address,undefined -o "$OUT/complete_bulletproof_test_asan" \
    $(for f in $DRV crv harness; do echo a_$f.o; done) -lcrypto
echo "built $OUT/complete_bulletproof_test_cpu, $OUT/complete_bulletproof_test_asan"
LIB="$(cd "$HERE/.." && pwd)/cudabulletproof_amd"
if [ -f "$LIB/libcudabulletproof_hip.so" ]; then
    gcc -O2 -fPIC -c "$HERE/ref/det_rand.c" -o det_rand.o
    $CXX -o "$OUT/complete_bulletproof_test_hip" $(for f in $DRV; do echo p_$f.o; done) det_rand.o \
        -L"$LIB" -lcudabulletproof_hip -Wl,-rpath,'$ORIGIN/../../cudabulletproof_amd' -lcrypto
    echo "built $OUT/complete_bulletproof_test_hip"
fi
