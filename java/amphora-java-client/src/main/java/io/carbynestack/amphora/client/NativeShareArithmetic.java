/*
 * MI355X-native share arithmetic for the Amphora client: the JNI entry points
 * of libamphora_jni (jni/amphora_jni.c) over libamphora_hip
 * (include/amphora.h), plus the BigInteger <-> 16-byte word packing the
 * boundary needs (SURVEY.md 8b: arbitrary BigIntegers are reduced mod p,
 * words are little-endian).
 *
 * Written for the reference tree (drop into amphora-java-client); no JDK
 * exists in the build image, so this file is compiled only by jni/Makefile
 * when a JDK and the reference's classpath are present.
 */
package io.carbynestack.amphora.client;

import java.math.BigInteger;
import java.util.ArrayList;
import java.util.List;

final class NativeShareArithmetic {
  static final int WORD_WIDTH = 16; // MpSpdzIntegrationUtils.WORD_WIDTH
  private static final BigInteger MASK128 = BigInteger.ONE.shiftLeft(128).subtract(BigInteger.ONE);

  static {
    System.loadLibrary("amphora_jni"); // libamphora_jni.so -> libamphora_hip.so
  }

  private NativeShareArithmetic() {}

  /** amph_ctx_create / amph_ctx_create_multi; devices null = device 0 */
  static native long ctxCreate(byte[] primeLe, byte[] rLe, byte[] rInvLe, int[] devices);

  static native void ctxDestroy(long ctx);

  /** verifyOutputDeliveryObjects: -1 if every word verified, else the smallest failing word */
  static native long recombineVerify(
      long ctx, byte[][] y, byte[][] r, byte[][] v, byte[][] w, byte[][] u, byte[] outSecretsLe);

  /** verify the Input Mask ODOs + maskInput for every secret word: -1 or the failing word */
  static native long maskInput(
      long ctx, byte[][] y, byte[][] r, byte[][] v, byte[][] w, byte[][] u, byte[] secretsLe,
      byte[] outMasked);

  /** recombineObject: canonical LE16 words */
  static native void recombine(long ctx, byte[][] shares, byte[] outLe);

  /** verifySecrets over canonical LE16 arrays (Java argument order): -1 or the failing word */
  static native long verify(long ctx, byte[] ys, byte[] rs, byte[] us, byte[] vs, byte[] ws);

  /** maskInput over canonical LE16 secrets and masks: toGfp((s - m) mod p) per word */
  static native void maskWords(long ctx, byte[] secretsLe, byte[] masksLe, byte[] outMasked);

  /**
   * maskInput for ONE word (SecretShareUtil.java:65-68): host arithmetic in libamphora_hip, no
   * kernel launch (amph_mask_word_host); the batch path is maskInput above
   */
  static native byte[] maskWord(long ctx, byte[] secretLe, byte[] maskLe);

  static native String verifyMessage(long ctx, byte[] y, byte[] r, byte[] u, byte[] v, byte[] w);

  /** getSecret from the five base64 strings per party (ASCII): -1 or the failing word */
  static native long recombineVerifyB64(
      long ctx, byte[][] y, byte[][] r, byte[][] v, byte[][] w, byte[][] u, long words, byte[] outLe);

  /** createSecret from the /input-masks text: the 24-character MaskedInputData records */
  static native long maskInputB64(
      long ctx, byte[][] y, byte[][] r, byte[][] v, byte[][] w, byte[][] u, long words,
      byte[] secretsLe, byte[] outRecords24);

  /** LE16 of x mod p (x reduced only when negative or wider than 128 bits, as the kernels
   * canonicalise any 128-bit word themselves) */
  static void putWord(BigInteger x, BigInteger prime, byte[] out, int word) {
    BigInteger v = x.signum() < 0 || x.bitLength() > 128 ? x.mod(prime) : x;
    byte[] be = v.toByteArray(); // big-endian two's complement, maybe a leading 0
    int off = word * WORD_WIDTH;
    for (int k = 0; k < WORD_WIDTH; k++) {
      int i = be.length - 1 - k;
      out[off + k] = i >= 0 ? be[i] : 0;
    }
  }

  static byte[] le16(BigInteger x) {
    if (x.signum() < 0 || x.compareTo(MASK128) > 0) {
      throw new IllegalArgumentException("not a 128-bit unsigned integer: " + x);
    }
    byte[] out = new byte[WORD_WIDTH];
    putWord(x, null, out, 0);
    return out;
  }

  static byte[] pack(List<BigInteger> values, BigInteger prime) {
    byte[] out = new byte[values.size() * WORD_WIDTH];
    for (int i = 0; i < values.size(); i++) putWord(values.get(i), prime, out, i);
    return out;
  }

  static byte[] pack(BigInteger[] values, int count, BigInteger prime) {
    byte[] out = new byte[count * WORD_WIDTH];
    for (int i = 0; i < count; i++) putWord(values[i], prime, out, i);
    return out;
  }

  static BigInteger word(byte[] le, int word) {
    byte[] be = new byte[WORD_WIDTH];
    for (int k = 0; k < WORD_WIDTH; k++) be[k] = le[word * WORD_WIDTH + WORD_WIDTH - 1 - k];
    return new BigInteger(1, be);
  }

  static List<BigInteger> unpack(byte[] le, int words) {
    List<BigInteger> out = new ArrayList<>(words);
    for (int i = 0; i < words; i++) out.add(word(le, i));
    return out;
  }

  /** Devices from the system property amphora.gpu.devices ("0,1,..."), null = device 0 */
  static int[] devices() {
    String d = System.getProperty("amphora.gpu.devices", "").trim();
    if (d.isEmpty()) return null;
    String[] parts = d.split(",");
    int[] out = new int[parts.length];
    for (int i = 0; i < parts.length; i++) out[i] = Integer.parseInt(parts[i].trim());
    return out;
  }
}
