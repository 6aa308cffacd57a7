"""The JVM-side call-site changes as committed patches:
java/patches/*.patch against the reference sources the Java drop-ins serve.

* DefaultAmphoraClient.patch: createSecret (DefaultAmphoraClient.java:150-160)
  masks the whole secret with ONE SecretShareUtil.maskInputs call (verify +
  mask on the GPU) instead of the per-word parallel loop, and
  verifyOutputDeliveryObjects (:476-505) is ONE verifyOutputDeliveryObjects
  call instead of five recombineObject + verifySecrets;
* OutputDeliveryService.patch: computeOutputDeliveryObject (:75-161) runs
  NativeOutputDelivery.pre / post around the unchanged Castor downloads,
  operationId and open (every party's diffs are collected unsummed from the
  cache and summed on the GPU); multiplyShares (:176-229) keeps its BigInteger
  form for its package-private callers.

The test applies each patch to a scratch copy of the reference file (CPU
only; skipped where /root/reference is absent, e.g. on the GPU box) with
`patch -p1`, first as a dry run, and checks the patched file calls the
drop-in API that java/ defines (no JDK exists here to compile it).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCHES = os.path.join(ROOT, "java", "patches")

CASES = {
    "DefaultAmphoraClient.patch": (
        "amphora-java-client/src/main/java/io/carbynestack/amphora/client/DefaultAmphoraClient.java",
        ["secretShareUtil.maskInputs(secret.getData(), inputMaskOutputDeliveryObjects)",
         "return secretShareUtil.verifyOutputDeliveryObjects(outputDeliveryObjects);"],
        ["secretShareUtil.maskInput(", "secretShareUtil.recombineObject(", "secretShareUtil.verifySecrets("]),
    "OutputDeliveryService.patch": (
        "amphora-service/src/main/java/io/carbynestack/amphora/service/calculation/OutputDeliveryService.java",
        ["NativeOutputDelivery.pre(ctx, shareData, stride, inputMaskShares, tripleShares)",
         "NativeOutputDelivery.post(ctx, local, partyDiffs, amphoraProperties.getPlayerId() == 0)",
         "computeOutputDeliveryObject(secretShare.getData(), SHARE_WIDTH, requestId)",
         "private final SecretShareUtil secretShareUtil;",
         "List<FactorPair> recombineDiffs(UUID operationId)",
         "List<List<FactorPair>> collectDiffs(UUID operationId)"],
        []),
}


def java_methods(path):
    """static / instance method names a drop-in source declares."""
    src = open(path).read()
    return set(re.findall(r"\b(\w+)\s*\([^;{)]*\)\s*(?:throws [\w., ]+)?\{", src))


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent (GPU box)")
@pytest.mark.parametrize("name", sorted(CASES))
def test_patch_applies_to_reference(tmp_path, name):
    rel, must, gone = CASES[name]
    dst = tmp_path / rel
    dst.parent.mkdir(parents=True)
    shutil.copy(os.path.join(REF, rel), dst)
    patch = os.path.join(PATCHES, name)
    for extra in (["--dry-run"], []):
        r = subprocess.run(["patch", "-p1", "--batch", "--forward"] + extra + ["-i", patch],
                           cwd=tmp_path, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "offset" not in r.stdout and "fuzz" not in r.stdout, r.stdout  # applies exactly
    text = dst.read_text()
    for s in must:
        assert s in text, s
    for s in gone:
        assert s not in text, s
    assert not list(tmp_path.rglob("*.rej"))


def test_patched_calls_exist_in_the_dropins():
    """Every drop-in method the patches call is defined by java/."""
    client = java_methods(os.path.join(
        ROOT, "java/amphora-java-client/src/main/java/io/carbynestack/amphora/client/SecretShareUtil.java"))
    assert {"maskInputs", "verifyOutputDeliveryObjects", "maskInput"} <= client
    nod = java_methods(os.path.join(
        ROOT, "java/amphora-service/src/main/java/io/carbynestack/amphora/service/calculation/"
              "NativeOutputDelivery.java"))
    assert {"pre", "post", "diffs"} <= nod
    svc = java_methods(os.path.join(
        ROOT, "java/amphora-service/src/main/java/io/carbynestack/amphora/service/calculation/"
              "SecretShareUtil.java"))
    assert "context" in svc


def test_native_methods_match_jni_exports():
    """Each `static native` method of the two NativeShareArithmetic classes has
    a Java_<package>_NativeShareArithmetic_<name> entry point in
    jni/amphora_jni.c, and every entry point is declared in Java."""
    jni = open(os.path.join(ROOT, "jni", "amphora_jni.c")).read()
    exported = {("client", m) for m in re.findall(r"CLIENT\((\w+)\)", jni)} | \
               {("service", m) for m in re.findall(r"SERVICE\((\w+)\)", jni)}
    declared = set()
    for side, rel in (("client", "java/amphora-java-client/src/main/java/io/carbynestack/amphora/client/"
                                 "NativeShareArithmetic.java"),
                      ("service", "java/amphora-service/src/main/java/io/carbynestack/amphora/service/"
                                  "calculation/NativeShareArithmetic.java")):
        src = open(os.path.join(ROOT, rel)).read()
        declared |= {(side, m) for m in re.findall(r"static native [\w\[\]]+\s+(\w+)\s*\(", src)}
    exported.discard(("client", "name"))
    exported.discard(("service", "name"))
    assert declared == exported, (declared ^ exported)
