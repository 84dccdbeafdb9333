"""ChordKey: host-side value type mirroring the reference's key class.

GenericKey<16,32> (src/data_structures/key.h:56-281, ChordKey at key.h:355).
Values are held as raw uint256 integers so the reference's non-canonical
results survive (1 - 1 -> 2^128, 0 - 1 -> 2^256 - 1: key.h:242-250).
`in_between` and plaintext hashing are answered by the engine's GPU kernels
(cx_in_between, cx_uuid5_dns), the same code the batch API uses; this class
only builds, formats and does the reference's scalar +/- on values.
"""
from __future__ import annotations

import numpy as np

RING_BITS = 128
KEYS_IN_RING = 1 << RING_BITS  # 16^32, key.h:279-280
U256 = 1 << 256


class ChordKey:
    __slots__ = ("value", "plaintext")

    def __init__(self, key, hashed: bool = True):
        """ChordKey(str, hashed) (key.h:70-82) or ChordKey(int) (key.h:89-93)."""
        self.plaintext = ""
        if isinstance(key, str):
            if hashed:  # uint256_t("0x" + key), key.h:73-75
                self.value = int(key, 16) if key else 0
            else:  # UUIDv5(DNS, plaintext) read big-endian, key.h:76-79 (GPU)
                from .ring import uuid5_dns
                self.plaintext = key
                lo, hi = (int(x) for x in uuid5_dns([key])[0])
                self.value = lo | (hi << 64)
        else:
            self.value = int(key) % U256

    # IntToHexStr (key.h:41-47): lowercase, no leading zeros
    def __str__(self) -> str:
        return format(self.value, "x")

    def __repr__(self) -> str:
        return f"ChordKey({self})"

    def __int__(self) -> int:
        return self.value

    def __eq__(self, other) -> bool:
        return isinstance(other, ChordKey) and self.value == other.value

    def __lt__(self, other) -> bool:
        return self.value < other.value

    def __hash__(self) -> int:
        return hash(self.value)

    def __add__(self, other) -> "ChordKey":
        if isinstance(other, ChordKey):  # key.h:252-256
            return ChordKey((self.value + other.value) % KEYS_IN_RING)
        return ChordKey(((self.value + int(other)) % U256) % KEYS_IN_RING)  # key.h:236-240

    def __sub__(self, other) -> "ChordKey":
        if isinstance(other, ChordKey):  # key.h:258-270 (signed difference)
            d = self.value - other.value
        else:  # key.h:242-250 (uint256 difference, wraps)
            d = (self.value - int(other)) % U256
        return ChordKey(d if d > 0 else KEYS_IN_RING + d)

    def cx(self) -> tuple[int, int]:
        """(lo, hi) limbs of the canonical value (cx_u128)."""
        v = self.value % KEYS_IN_RING
        return v & 0xFFFFFFFFFFFFFFFF, v >> 64

    def in_between(self, lower_bound, upper_bound, inclusive: bool = True) -> bool:
        """InBetween (key.h:103-131), evaluated by the engine (GPU)."""
        from .ring import in_between

        def u256(x):
            v = int(x) % U256
            return [(v >> (64 * j)) & 0xFFFFFFFFFFFFFFFF for j in range(4)]

        arr = lambda x: np.array([u256(x)], dtype=np.uint64)  # noqa: E731
        return bool(in_between(arr(self), arr(lower_bound), arr(upper_bound), inclusive)[0])

    @staticmethod
    def array(keys) -> np.ndarray:
        """(q, 2) uint64 array (lo, hi) of ChordKeys / ints / hex strings."""
        out = np.empty((len(keys), 2), dtype=np.uint64)
        for i, k in enumerate(keys):
            v = k.value if isinstance(k, ChordKey) else (int(k, 16) if isinstance(k, str) else int(k))
            v %= KEYS_IN_RING
            out[i, 0] = v & 0xFFFFFFFFFFFFFFFF
            out[i, 1] = v >> 64
        return out

    @staticmethod
    def array_plaintext(names) -> np.ndarray:
        """(q, 2) uint64 IDs of plaintext names, hashed in one GPU batch."""
        from .ring import uuid5_dns
        return uuid5_dns(list(names))

    @staticmethod
    def from_array(a) -> list:
        a = np.asarray(a, dtype=np.uint64).reshape(-1, 2)
        return [ChordKey(int(lo) | (int(hi) << 64)) for lo, hi in a]
