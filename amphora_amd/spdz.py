"""SPDZ field parameters of the reference's test and default deployments.

The prime, the Montgomery auxiliary modulus r = 2^128 mod p and its inverse
are configuration in the reference, not code: amphora-service's
application-test.properties:36-38 (SPDZ_PRIME / SPDZ_R / SPDZ_R_INV) and the
client tests (amphora-java-client/.../SecretShareUtilTest.java:24-28) use
these values.  They live here so product-side callers (bench.py, tools)
never reach into oracle/, which is test infrastructure.
"""
TEST_PRIME = 198766463529478683931867765928436695041  # 0x958907458f2136861bd7554a24340001
TEST_R = 141515903391459779531506841503331516415      # 2^128 mod p
TEST_RINV = 133854242216446749056083838363708373830   # r^-1 mod p

assert TEST_R == (1 << 128) % TEST_PRIME and TEST_R * TEST_RINV % TEST_PRIME == 1
