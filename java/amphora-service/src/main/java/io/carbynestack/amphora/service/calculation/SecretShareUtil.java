/*
 * Drop-in for amphora-service's SecretShareUtil (calculation/SecretShareUtil.java:30-107)
 * whose per-word arithmetic runs on an MI355X through libamphora_hip: same
 * constructor (the @Bean of UtilsConfig.java:22-25 keeps working), same
 * convertToSecretShare contract and message.
 *
 * Unbuildable in this image (no JDK): compiled by jni/Makefile against the
 * reference's classpath when one is present.
 */
package io.carbynestack.amphora.service.calculation;

import static org.springframework.util.Assert.isTrue;

import io.carbynestack.amphora.common.MaskedInput;
import io.carbynestack.amphora.common.MaskedInputData;
import io.carbynestack.amphora.common.SecretShare;
import io.carbynestack.castor.common.entities.Field;
import io.carbynestack.castor.common.entities.InputMask;
import io.carbynestack.castor.common.entities.Share;
import io.carbynestack.castor.common.entities.TupleList;
import io.carbynestack.mpspdz.integration.MpSpdzIntegrationUtils;
import java.math.BigInteger;
import java.util.List;
import org.springframework.beans.factory.annotation.Autowired;

public class SecretShareUtil implements AutoCloseable {
  static final int WORD_WIDTH = 16; // MpSpdzIntegrationUtils.WORD_WIDTH

  private final BigInteger prime;
  private long ctx;

  @Autowired
  public SecretShareUtil(MpSpdzIntegrationUtils spdzUtil) {
    this.prime = spdzUtil.getPrime();
    this.ctx = createContext(spdzUtil);
  }

  /**
   * The context for the CONFIGURED field (UtilsConfig.java:17-20: SpdzProperties prime, r, rInv):
   * r and rInv are read back from the configured codec itself -- toGfp(1) = r mod p and
   * fromGfp(word 1) = rInv mod p under the Montgomery encoding -- not recomputed, so a deployment
   * whose r is not 2^128 mod p is refused by amph_ctx_create ("r must equal 2^128 mod prime")
   * instead of silently diverging from the reference.
   */
  static long createContext(MpSpdzIntegrationUtils spdzUtil) {
    BigInteger prime = spdzUtil.getPrime();
    byte[] one = new byte[WORD_WIDTH];
    one[0] = 1;
    BigInteger r = leInt(spdzUtil.toGfp(BigInteger.ONE));
    BigInteger rInv = spdzUtil.fromGfp(one);
    return NativeShareArithmetic.ctxCreate(le16(prime), le16(r), le16(rInv), devices());
  }

  static BigInteger leInt(byte[] le) {
    byte[] be = new byte[le.length];
    for (int k = 0; k < le.length; k++) be[k] = le[le.length - 1 - k];
    return new BigInteger(1, be);
  }

  @Override
  public synchronized void close() {
    if (ctx != 0) {
      NativeShareArithmetic.ctxDestroy(ctx);
      ctx = 0;
    }
  }

  long context() {
    return ctx;
  }

  /**
   * Converts a given {@link MaskedInput} to this party's {@link SecretShare} (:58-81): per word,
   * value' = [mask value] + (useZeroInputAsData ? 0 : [masked]) and mac' = [mask mac] + key *
   * masked, mod p, as 32-byte value || mac.
   *
   * @throws IllegalArgumentException "Received more input data than available inputMasks." when
   *     the counts differ
   */
  public SecretShare convertToSecretShare(
      MaskedInput maskedInput,
      String macKey,
      TupleList<InputMask<Field.Gfp>, Field.Gfp> inputMask,
      boolean useZeroInputAsData) {
    List<MaskedInputData> data = maskedInput.getData();
    isTrue(data.size() == inputMask.size(), "Received more input data than available inputMasks.");
    int words = data.size();
    byte[] masked = new byte[words * WORD_WIDTH];
    byte[] tuples = new byte[words * 2 * WORD_WIDTH];
    for (int i = 0; i < words; i++) {
      System.arraycopy(data.get(i).getValue(), 0, masked, i * WORD_WIDTH, WORD_WIDTH);
      Share s = inputMask.get(i).getShare(0);
      System.arraycopy(s.getValue(), 0, tuples, 2 * i * WORD_WIDTH, WORD_WIDTH);
      System.arraycopy(s.getMac(), 0, tuples, (2 * i + 1) * WORD_WIDTH, WORD_WIDTH);
    }
    byte[] out = new byte[words * 2 * WORD_WIDTH];
    NativeShareArithmetic.convertShare(
        ctx, masked, tuples, le16(new BigInteger(macKey).mod(prime)), useZeroInputAsData, out);
    return SecretShare.builder()
        .secretId(maskedInput.getSecretId())
        .data(out)
        .tags(maskedInput.getTags())
        .build();
  }

  static byte[] le16(BigInteger x) {
    byte[] be = x.toByteArray();
    byte[] out = new byte[WORD_WIDTH];
    for (int k = 0; k < WORD_WIDTH; k++) {
      int i = be.length - 1 - k;
      out[k] = i >= 0 ? be[i] : 0;
    }
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
