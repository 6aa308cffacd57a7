/*
 * The local arithmetic of OutputDeliveryService (OutputDeliveryService.java:100-286)
 * on an MI355X, for the three places it is used (INTEGRATION.md section 2):
 *
 *   Local l = NativeOutputDelivery.pre(ctx, shareData, 32, masks, triples);
 *       // computeOutputDeliveryObject :100-139 + multiplyShares' diffs :186-200
 *       // (the triples are downloaded before the diffs; operationId only needs 2W)
 *   new MultiplicationExchangeObject(operationId, playerId, l.diffs())  // unchanged open
 *   byte[][] wu = NativeOutputDelivery.post(ctx, l, allPartiesDiffs, playerId == 0);
 *       // recombineDiffs :231-272 + multiplySharedSecrets :274-286 + toGfp :147-152
 *   OutputDeliveryObject.builder().secretShares(l.y).rShares(l.r).vShares(l.v)
 *       .wShares(wu[0]).uShares(wu[1]).build();
 *
 * The signed diffs cross the open as FactorPairs of BigIntegers exactly as in
 * the reference (unreduced x - a, |x - a| < p), so partners running the Java
 * path interoperate.
 *
 * Session (the device-resident form, INTEGRATION.md section 2): the triples,
 * every party's diffs and the ODO fields stay on the GPU between the steps and
 * only the texts cross PCIe (72 vs 132-170 ms for 4 Mi words x 3 parties,
 * DESIGN.md "Round 3 in brief"):
 *
 *   try (Session s = new Session(ctx, shareData, 32, masks, triples, nParties, false)) {
 *     byte[] interim = s.interimValuesText();      // the JSON array of this party's FactorPairs
 *     // ... send it inside its MultiplicationExchangeObject, receive each partner's body ...
 *     s.partner(slot, body, off, len);             // slot 1..nParties-1, the array's span
 *     byte[][] odoB64 = s.finishBase64(playerId == 0);  // secretShares .. uShares as base64
 *   }
 *
 * Unbuildable in this image (no JDK).
 */
package io.carbynestack.amphora.service.calculation;

import io.carbynestack.amphora.common.FactorPair;
import io.carbynestack.castor.common.entities.Field;
import io.carbynestack.castor.common.entities.InputMask;
import io.carbynestack.castor.common.entities.MultiplicationTriple;
import io.carbynestack.castor.common.entities.Share;
import io.carbynestack.castor.common.entities.TupleList;
import java.math.BigInteger;
import java.util.ArrayList;
import java.util.List;

final class NativeOutputDelivery {
  private static final int W16 = SecretShareUtil.WORD_WIDTH;

  private NativeOutputDelivery() {}

  /** One party's ODO front half and its own signed diffs (2 FactorPairs per word). */
  static final class Local {
    final byte[] y;
    final byte[] r;
    final byte[] v;
    final byte[] diffMag; // 32 B per FactorPair: |a| || |b|, little-endian
    final byte[] diffNeg; // 2 B per FactorPair: a < 0, b < 0
    final byte[] triples; // the castor stream, 96 B per triple, kept for post()

    Local(int words, byte[] triples) {
      y = new byte[words * W16];
      r = new byte[words * W16];
      v = new byte[words * W16];
      diffMag = new byte[words * 4 * W16];
      diffNeg = new byte[words * 4];
      this.triples = triples;
    }

    /** the FactorPairs the reference puts into its MultiplicationExchangeObject */
    List<FactorPair> diffs() {
      int pairs = diffNeg.length / 2;
      List<FactorPair> out = new ArrayList<>(pairs);
      for (int i = 0; i < pairs; i++) {
        out.add(FactorPair.of(signed(diffMag, 2 * i, diffNeg[2 * i]), signed(diffMag, 2 * i + 1, diffNeg[2 * i + 1])));
      }
      return out;
    }
  }

  /** shareData: SecretShare.data (stride 32) or raw words (stride 16); 2W masks, 2W triples */
  static Local pre(
      long ctx,
      byte[] shareData,
      int stride,
      TupleList<InputMask<Field.Gfp>, Field.Gfp> masks,
      TupleList<MultiplicationTriple<Field.Gfp>, Field.Gfp> triples) {
    int words = shareData.length / stride;
    byte[] m = new byte[masks.size() * 2 * W16];
    for (int i = 0; i < masks.size(); i++) put(masks.get(i).getShare(0), m, 2 * i);
    byte[] t = new byte[triples.size() * 6 * W16];
    for (int i = 0; i < triples.size(); i++) {
      for (int k = 0; k < 3; k++) put(triples.get(i).getShare(k), t, 6 * i + 2 * k);
    }
    Local l = new Local(words, t);
    NativeShareArithmetic.odoPre(ctx, shareData, stride, m, t, l.y, l.r, l.v, l.diffMag, l.diffNeg);
    return l;
  }

  /**
   * @param partyDiffs every party's FactorPairs, this party's included (recombineDiffs sums
   *     rangeClosed(0, vcPartners.size()))
   * @return {wShares, uShares}
   */
  static byte[][] post(long ctx, Local own, List<List<FactorPair>> partyDiffs, boolean isPlayer0) {
    int n = partyDiffs.size();
    byte[][] mags = new byte[n][];
    byte[][] negs = new byte[n][];
    for (int j = 0; j < n; j++) {
      List<FactorPair> d = partyDiffs.get(j);
      mags[j] = new byte[d.size() * 2 * W16];
      negs[j] = new byte[d.size() * 2];
      for (int i = 0; i < d.size(); i++) {
        unsigned(d.get(i).getA(), mags[j], negs[j], 2 * i);
        unsigned(d.get(i).getB(), mags[j], negs[j], 2 * i + 1);
      }
    }
    byte[][] wu = {new byte[own.y.length], new byte[own.y.length]};
    NativeShareArithmetic.openPost(ctx, mags, negs, own.triples, isPlayer0, wu[0], wu[1]);
    return wu;
  }

  /** One request's Output Delivery with device-resident state (amph_party_*). */
  static final class Session implements AutoCloseable {
    private long handle;
    final int words;
    final byte[] y; // null unless withFields
    final byte[] r;
    final byte[] v;

    /**
     * @param withFields fill y, r, v here (for finish()); false leaves them on the GPU for
     *     finishBase64()
     */
    Session(
        long ctx,
        byte[] shareData,
        int stride,
        TupleList<InputMask<Field.Gfp>, Field.Gfp> masks,
        TupleList<MultiplicationTriple<Field.Gfp>, Field.Gfp> triples,
        int nParties,
        boolean withFields) {
      words = shareData.length / stride;
      byte[] m = new byte[masks.size() * 2 * W16];
      for (int i = 0; i < masks.size(); i++) put(masks.get(i).getShare(0), m, 2 * i);
      byte[] t = new byte[triples.size() * 6 * W16];
      for (int i = 0; i < triples.size(); i++) {
        for (int k = 0; k < 3; k++) put(triples.get(i).getShare(k), t, 6 * i + 2 * k);
      }
      y = withFields ? new byte[words * W16] : null;
      r = withFields ? new byte[words * W16] : null;
      v = withFields ? new byte[words * W16] : null;
      handle = NativeShareArithmetic.partyBegin(ctx, shareData, stride, m, t, nParties, y, r, v);
    }

    /** this party's MultiplicationExchangeObject.interimValues, as the JSON array Jackson writes */
    byte[] interimValuesText() {
      return NativeShareArithmetic.partyText(handle);
    }

    /** a partner's interimValues: body[off, off + len) is its JSON array */
    void partner(int slot, byte[] body, int off, int len) {
      NativeShareArithmetic.partyPartner(handle, slot, body, off, len);
    }

    /** @return {wShares, uShares} */
    byte[][] finish(boolean isPlayer0) {
      byte[][] wu = {new byte[words * W16], new byte[words * W16]};
      NativeShareArithmetic.partyFinish(handle, isPlayer0, wu[0], wu[1]);
      return wu;
    }

    /** @return the five ODO fields (secretShares, rShares, vShares, wShares, uShares) as base64 */
    byte[][] finishBase64(boolean isPlayer0) {
      int chars = 4 * ((words * W16 + 2) / 3);
      byte[][] f = new byte[5][chars];
      NativeShareArithmetic.partyFinishBase64(handle, isPlayer0, f);
      return f;
    }

    @Override
    public synchronized void close() {
      if (handle != 0) {
        NativeShareArithmetic.partyFree(handle);
        handle = 0;
      }
    }
  }

  private static void put(Share s, byte[] out, int word) {
    System.arraycopy(s.getValue(), 0, out, word * W16, W16);
    System.arraycopy(s.getMac(), 0, out, (word + 1) * W16, W16);
  }

  private static BigInteger signed(byte[] mag, int value, byte neg) {
    byte[] be = new byte[W16];
    for (int k = 0; k < W16; k++) be[k] = mag[value * W16 + W16 - 1 - k];
    BigInteger x = new BigInteger(1, be);
    return neg != 0 ? x.negate() : x;
  }

  private static void unsigned(BigInteger x, byte[] mag, byte[] neg, int value) {
    neg[value] = (byte) (x.signum() < 0 ? 1 : 0);
    byte[] be = x.abs().toByteArray();
    if (be.length > W16 + 1 || (be.length == W16 + 1 && be[0] != 0)) {
      throw new IllegalArgumentException("interim value wider than 128 bits: " + x);
    }
    for (int k = 0; k < W16; k++) {
      int i = be.length - 1 - k;
      mag[value * W16 + k] = i >= 0 ? be[i] : 0;
    }
  }
}
