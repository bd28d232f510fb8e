"""liblcb_amd — MI355X-native batch digest engine for liblcb's crypto/hash path.

The product is the C-ABI library liblcb_hash_gpu.so (include/lcb_hash_gpu.h,
HIP kernels in csrc/).  This package is its host-side Python mirror of the
reference's one-shot API (liblcb_amd.hash), the CRC-32 family of
include/math/crc32.h (liblcb_amd.crc32), the ChaCha / XChaCha cipher of
include/crypto/cipher/chacha.h (liblcb_amd.chacha), the asynchronous
packet ingestion queue (liblcb_amd.queue) and batched RADIUS packet
signing / verification over the keyed batches (liblcb_amd.radius).
"""
from ._lib import (ALG_IDS, ALG_NAMES, BLOCK_SIZE, DIGEST_SIZE, GOST256, GOST512, MD5, SHA1,
                   SHA224, SHA256, SHA384, SHA512, LcbHashError, lib)
from .hash import *  # noqa: F401,F403
from . import chacha, crc32, queue, radius  # noqa: F401,E402  (cipher, CRC-32, ingestion queue, RADIUS)

__all__ = ["ALG_IDS", "ALG_NAMES", "BLOCK_SIZE", "DIGEST_SIZE", "MD5", "SHA1", "SHA224",
           "SHA256", "SHA384", "SHA512", "GOST256", "GOST512", "LcbHashError", "lib"]
