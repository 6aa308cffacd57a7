/*
 * Drop-in for amphora-java-client's SecretShareUtil (SecretShareUtil.java:33-157)
 * whose arithmetic runs on an MI355X through libamphora_hip: same package,
 * same package-private API and static factory of(prime, r, rInv) (which
 * DefaultAmphoraClientTest mocks statically, DefaultAmphoraClientTest.java:114-118),
 * same exceptions and messages.  Two batch entry points are added for
 * DefaultAmphoraClient (INTEGRATION.md section 1): verifyOutputDeliveryObjects
 * (:476-505, the five recombineObject calls + verifySecrets in one launch) and
 * maskInputs (createSecret :150-160, verify + mask in one launch).
 *
 * Unbuildable in this image (no JDK): compiled by jni/Makefile against the
 * reference's classpath when one is present.
 */
package io.carbynestack.amphora.client;

import static io.carbynestack.amphora.client.NativeShareArithmetic.WORD_WIDTH;

import io.carbynestack.amphora.common.MaskedInputData;
import io.carbynestack.amphora.common.OutputDeliveryObject;
import io.carbynestack.amphora.common.exceptions.IntegrityVerificationException;
import java.math.BigInteger;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.List;
import lombok.Getter;
import lombok.NonNull;

class SecretShareUtil implements AutoCloseable {
  @Getter @NonNull private final BigInteger prime;
  @Getter @NonNull private final BigInteger r;
  @Getter @NonNull private final BigInteger rInv;
  private long ctx;

  private SecretShareUtil(BigInteger prime, BigInteger r, BigInteger rInv, long ctx) {
    this.prime = prime;
    this.r = r;
    this.rInv = rInv;
    this.ctx = ctx;
  }

  /**
   * Creates a new {@link SecretShareUtil} on the GPU(s) named by the system property
   * amphora.gpu.devices (default: device 0).
   *
   * @throws NullPointerException if any of the parameters is <i>null</i>
   * @throws IllegalArgumentException if r is not 2^128 mod prime or rInv not its inverse
   */
  static SecretShareUtil of(
      @NonNull BigInteger prime, @NonNull BigInteger r, @NonNull BigInteger rInv) {
    long ctx =
        NativeShareArithmetic.ctxCreate(
            NativeShareArithmetic.le16(prime),
            NativeShareArithmetic.le16(r),
            NativeShareArithmetic.le16(rInv),
            NativeShareArithmetic.devices());
    return new SecretShareUtil(prime, r, rInv, ctx);
  }

  @Override
  public synchronized void close() {
    if (ctx != 0) {
      NativeShareArithmetic.ctxDestroy(ctx);
      ctx = 0;
    }
  }

  /**
   * maskInput :65-68: MaskedInputData.of(toGfp((secret - inputMask) mod p)).
   *
   * <p>One word: computed on the calling thread (amph_mask_word_host), with no kernel launch and
   * no stream synchronisation, so the unpatched DefaultAmphoraClient's per-word parallel loop
   * (:155-160) costs what the BigInteger code did. The GPU path for a whole secret is {@link
   * #maskInputs} (java/patches/DefaultAmphoraClient.patch).
   */
  MaskedInputData maskInput(BigInteger secret, BigInteger inputMask) {
    byte[] s = new byte[WORD_WIDTH];
    byte[] m = new byte[WORD_WIDTH];
    NativeShareArithmetic.putWord(secret, prime, s, 0);
    NativeShareArithmetic.putWord(inputMask, prime, m, 0);
    return MaskedInputData.of(NativeShareArithmetic.maskWord(ctx, s, m));
  }

  /**
   * recombineObject :70-90: word i = sum over the shares of fromGfp(word i) mod p. The word count
   * is shares.get(0).length / 16 and the other parties' arrays keep the reference's
   * Arrays.copyOfRange semantics (longer: cut; ending inside the last word: zero-padded; shorter
   * than that: ArrayIndexOutOfBoundsException) -- amph_recombine_object, INTEGRATION.md.
   */
  List<BigInteger> recombineObject(List<byte[]> shares) {
    if (shares.isEmpty()) {
      return new ArrayList<>();
    }
    int words = shares.get(0).length / WORD_WIDTH;
    byte[] out = new byte[words * WORD_WIDTH];
    NativeShareArithmetic.recombine(ctx, shares.toArray(new byte[0][]), out);
    return NativeShareArithmetic.unpack(out, words);
  }

  /**
   * verifySecrets :102-141: w_i == y_i r_i and u_i == v_i r_i (mod p) for every word.
   *
   * @throws IntegrityVerificationException for the smallest failing word, with the reference's
   *     message
   */
  void verifySecrets(
      List<BigInteger> secrets,
      List<BigInteger> rs,
      List<BigInteger> us,
      List<BigInteger> vs,
      List<BigInteger> ws) {
    int n = secrets.size();
    // a w or u outside [0, p) never equals a reduced product: fails on the host, and a
    // zero placeholder goes to the device so the other words are still checked
    int pre = n;
    List<BigInteger> w2 = new ArrayList<>(ws.subList(0, n));
    List<BigInteger> u2 = new ArrayList<>(us.subList(0, n));
    for (int i = 0; i < n; i++) {
      if (!inField(ws.get(i)) || !inField(us.get(i))) {
        if (pre == n) pre = i;
        w2.set(i, BigInteger.ZERO);
        u2.set(i, BigInteger.ZERO);
      }
    }
    long fail =
        NativeShareArithmetic.verify(
            ctx,
            NativeShareArithmetic.pack(secrets.subList(0, n), prime),
            NativeShareArithmetic.pack(rs.subList(0, n), prime),
            NativeShareArithmetic.pack(u2, prime),
            NativeShareArithmetic.pack(vs.subList(0, n), prime),
            NativeShareArithmetic.pack(w2, prime));
    int bad = fail >= 0 ? (int) Math.min(fail, pre) : pre;
    if (bad < n) {
      throw new IntegrityVerificationException(
          failureMessage(secrets.get(bad), rs.get(bad), us.get(bad), vs.get(bad), ws.get(bad)));
    }
  }

  /**
   * DefaultAmphoraClient.verifyOutputDeliveryObjects :476-505 in one launch: recombine the five
   * ODO fields over the parties and verify every word's MACs.
   *
   * @return the canonical secrets
   * @throws IntegrityVerificationException for the smallest failing word
   */
  List<BigInteger> verifyOutputDeliveryObjects(List<OutputDeliveryObject> odos) {
    if (odos.isEmpty()) {
      return new ArrayList<>();
    }
    byte[][][] f = fields(odos);
    int words = f[0][0].length / WORD_WIDTH;
    byte[] out = new byte[words * WORD_WIDTH];
    long fail = NativeShareArithmetic.recombineVerify(ctx, f[0], f[1], f[2], f[3], f[4], out);
    if (fail >= 0) {
      throw failureAt(f, (int) fail);
    }
    return NativeShareArithmetic.unpack(out, words);
  }

  /**
   * createSecret :150-160 in one launch: verify the Input Mask ODOs (all of them, as
   * verifyOutputDeliveryObjects does) and mask every secret word.
   *
   * @throws IntegrityVerificationException for the smallest failing mask word
   * @throws IndexOutOfBoundsException if the secret has more words than masks (after the masks
   *     verified, as inputMasks.get(i) fails in the reference)
   */
  List<MaskedInputData> maskInputs(BigInteger[] secret, List<OutputDeliveryObject> maskOdos) {
    if (maskOdos.isEmpty()) {
      if (secret.length > 0) throw new IndexOutOfBoundsException("Index 0 out of bounds for length 0");
      return new ArrayList<>();
    }
    byte[][][] f = fields(maskOdos);
    int words = f[0][0].length / WORD_WIDTH;
    if (secret.length > words) {
      verifyOutputDeliveryObjects(maskOdos);
      throw new IndexOutOfBoundsException(
          "Index " + words + " out of bounds for length " + words);
    }
    byte[] out = new byte[secret.length * WORD_WIDTH];
    long fail =
        NativeShareArithmetic.maskInput(
            ctx, f[0], f[1], f[2], f[3], f[4],
            NativeShareArithmetic.pack(secret, secret.length, prime), out);
    if (fail >= 0) {
      throw failureAt(f, (int) fail);
    }
    List<MaskedInputData> masked = new ArrayList<>(secret.length);
    for (int i = 0; i < secret.length; i++) {
      masked.add(MaskedInputData.of(Arrays.copyOfRange(out, i * WORD_WIDTH, (i + 1) * WORD_WIDTH)));
    }
    return masked;
  }

  private boolean inField(BigInteger x) {
    return x.signum() >= 0 && x.compareTo(prime) < 0;
  }

  /** the message of SecretShareUtil.java:116-129; the two products for this one word only */
  String failureMessage(BigInteger y, BigInteger r, BigInteger u, BigInteger v, BigInteger w) {
    BigInteger actualW = y.multiply(r).mod(prime);
    BigInteger actualU = v.multiply(r).mod(prime);
    return String.format(
        "Verification of secret has failed:%n"
            + "\t%s = %s * %s   &&   %s = %s * %s%n"
            + "\t%s = %s   &&   %s = %s",
        w, y, r, u, v, r, w, actualW, u, actualU);
  }

  // word i of every field, recombined over the parties -> the reference's message
  private IntegrityVerificationException failureAt(byte[][][] f, int i) {
    BigInteger[] x = new BigInteger[5];
    for (int k = 0; k < 5; k++) {
      List<byte[]> word = new ArrayList<>(f[k].length);
      for (byte[] party : f[k]) word.add(Arrays.copyOfRange(party, i * WORD_WIDTH, (i + 1) * WORD_WIDTH));
      x[k] = recombineObject(word).get(0);
    }
    // fields: y, r, v, w, u
    return new IntegrityVerificationException(failureMessage(x[0], x[1], x[4], x[2], x[3]));
  }

  private static byte[][][] fields(List<OutputDeliveryObject> odos) {
    int n = odos.size();
    byte[][][] f = new byte[5][n][];
    for (int j = 0; j < n; j++) {
      OutputDeliveryObject o = odos.get(j);
      f[0][j] = o.getSecretShares();
      f[1][j] = o.getRShares();
      f[2][j] = o.getVShares();
      f[3][j] = o.getWShares();
      f[4][j] = o.getUShares();
    }
    return f;
  }
}
