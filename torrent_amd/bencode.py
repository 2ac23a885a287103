"""Bencode codec, mirroring reference bencode.ts (used to read `info.pieces` and file lists).

Behaviour kept from the reference:
* decoded byte strings are views into the input (bencode.ts:104 `subarray`) -> memoryview;
* dict keys are decoded to text (bencode.ts:144-146), values stay bytes;
* the encoder writes dict keys in insertion order, NOT sorted (bencode.ts:56-64), and
  skips `None` values (bencode.ts:59 `val !== undefined`).
Malformed input raises ValueError (bencode.ts throws `Error("Failed to bdecode ...")`).
"""
from __future__ import annotations

from typing import Any

_COLON, _INT, _LIST, _DICT, _END = ord(":"), ord("i"), ord("l"), ord("d"), ord("e")


def _decode_int(data: memoryview, start: int):
    # bencode.ts:76-90
    if data[start] != _INT:
        raise ValueError("Failed to bdecode. Malformed int")
    end = start + 1
    n = len(data)
    while end < n and data[end] != _END:
        end += 1
    if end >= n:
        raise ValueError("Failed to bdecode. Malformed int")
    return end + 1, int(bytes(data[start + 1:end]).decode())


def _decode_str(data: memoryview, start: int):
    # bencode.ts:92-104
    ind = start
    n = len(data)
    while ind < n and data[ind] != _COLON:
        ind += 1
    if ind >= n:
        raise ValueError("Failed to bdecode. Malformed string")
    try:
        length = int(bytes(data[start:ind]).decode())
    except ValueError:
        raise ValueError("Failed to bdecode. Malformed string") from None
    if length < 0:  # an over-long length truncates, like subarray() (bencode.ts:103)
        raise ValueError("Failed to bdecode. Malformed string")
    return ind + length + 1, data[ind + 1:ind + 1 + length]


def _decode(data: memoryview, start: int):
    if start >= len(data):
        raise ValueError("Failed to bdecode. Unexpected end of input")
    c = data[start]
    if c == _DICT:
        out = {}
        n = start + 1
        while n < len(data) and data[n] != _END:
            n, key = _decode_str(data, n)
            n, val = _decode(data, n)
            out[bytes(key).decode("utf-8", "replace")] = val
        if n >= len(data):
            raise ValueError("Failed to bdecode. Malformed dictionary")
        return n + 1, out
    if c == _LIST:
        out = []
        n = start + 1
        while n < len(data) and data[n] != _END:
            n, val = _decode(data, n)
            out.append(val)
        if n >= len(data):
            raise ValueError("Failed to bdecode. Malformed list")
        return n + 1, out
    if c == _INT:
        return _decode_int(data, start)
    return _decode_str(data, start)


def bdecode(data) -> Any:
    """Decode bencoded bytes (bencode.ts:164).  Strings come back as memoryview slices."""
    mv = memoryview(data)
    return _decode(mv, 0)[1]


def _encode(out: bytearray, v: Any) -> None:
    if isinstance(v, str):
        b = v.encode()
        out += str(len(b)).encode() + b":" + b
    elif isinstance(v, (bytes, bytearray, memoryview)):
        b = bytes(v)
        out += str(len(b)).encode() + b":" + b
    elif isinstance(v, bool):
        raise TypeError("bool is not bencodeable")
    elif isinstance(v, int):
        out += b"i%de" % v
    elif isinstance(v, (list, tuple)):
        out.append(_LIST)
        for x in v:
            _encode(out, x)
        out.append(_END)
    elif isinstance(v, dict):
        out.append(_DICT)
        for k, x in v.items():  # insertion order (bencode.ts:56-64)
            if x is None:
                continue
            _encode(out, k)
            _encode(out, x)
        out.append(_END)
    else:
        raise TypeError(f"not bencodeable: {type(v)!r}")


def bencode(v: Any) -> bytes:
    """Encode (bencode.ts:71)."""
    out = bytearray()
    _encode(out, v)
    return bytes(out)
