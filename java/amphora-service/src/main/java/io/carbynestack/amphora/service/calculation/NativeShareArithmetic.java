/*
 * MI355X-native share arithmetic for amphora-service: the JNI entry points
 * of libamphora_jni (jni/amphora_jni.c) over libamphora_hip
 * (include/amphora.h).  Used by the SecretShareUtil drop-in and by
 * NativeOutputDelivery (the local parts of OutputDeliveryService).
 *
 * Written for the reference tree; no JDK exists in the build image, so this
 * file is compiled only by jni/Makefile when a JDK and the reference's
 * classpath are present.
 */
package io.carbynestack.amphora.service.calculation;

final class NativeShareArithmetic {
  static {
    System.loadLibrary("amphora_jni"); // libamphora_jni.so -> libamphora_hip.so
  }

  private NativeShareArithmetic() {}

  static native long ctxCreate(byte[] primeLe, byte[] rLe, byte[] rInvLe, int[] devices);

  static native void ctxDestroy(long ctx);

  /**
   * convertToSecretShare :58-107: maskedLe 16 B per word, maskTuples 32 B per word (value ||
   * mac of share 0), macKeyLe the party's MAC key mod p -> SecretShare.data (32 B per word)
   */
  static native void convertShare(
      long ctx, byte[] masked, byte[] maskTuples, byte[] macKeyLe, boolean useZeroInputAsData,
      byte[] outShare);

  /**
   * computeOutputDeliveryObject :100-139 + the local diffs of multiplyShares :186-200: y, r, v
   * (16 B per word) and the signed diffs (2 pairs per word: 64 B of magnitudes, 4 sign bytes)
   */
  static native void odoPre(
      long ctx, byte[] shareData, int stride, byte[] maskTuples, byte[] tripleTuples, byte[] y,
      byte[] r, byte[] v, byte[] diffMag, byte[] diffNeg);

  /** recombineDiffs :231-272 + multiplySharedSecrets :274-286 + the w/u encoding :147-152 */
  static native void openPost(
      long ctx, byte[][] diffMags, byte[][] diffNegs, byte[] tripleTuples, boolean isPlayer0,
      byte[] w, byte[] u);

  /** the interimValues array text Jackson writes for these diffs */
  static native byte[] exchangeEncode(long ctx, byte[] diffMag, byte[] diffNeg);

  /** body[off, off + len) = an interimValues array -> the signed diffs of npairs FactorPairs */
  static native void exchangeDecode(
      long ctx, byte[] body, int off, int len, long npairs, byte[] diffMag, byte[] diffNeg);

  /*
   * One request's Output Delivery with its triples, diffs and ODO fields kept on the GPU between
   * the steps (amph_party_*, include/amphora.h); see NativeOutputDelivery.Session.
   */

  /** tuples in, y/r/v out (or null: finishBase64 returns them) -> a session handle */
  static native long partyBegin(
      long ctx, byte[] shareData, int stride, byte[] maskTuples, byte[] tripleTuples, int nParties,
      byte[] y, byte[] r, byte[] v);

  /** this party's interimValues array text */
  static native byte[] partyText(long session);

  /** partner slot 1..nParties-1: body[off, off + len) = its interimValues array */
  static native void partyPartner(long session, int slot, byte[] body, int off, int len);

  /** w, u (16 B per word) */
  static native void partyFinish(long session, boolean isPlayer0, byte[] w, byte[] u);

  /** fields[0..4] = base64 (ASCII) of secretShares, rShares, vShares, wShares, uShares */
  static native void partyFinishBase64(long session, boolean isPlayer0, byte[][] fields);

  static native void partyFree(long session);
}
