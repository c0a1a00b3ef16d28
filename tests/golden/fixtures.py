"""Loaders for the golden fixtures written by make_golden.py."""
import base64
import json
import os
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))


def unhex(s: str) -> bytes:
    if s.startswith("z:"):
        return zlib.decompress(base64.b64decode(s[2:]))
    return bytes.fromhex(s)


def load(name: str):
    with open(os.path.join(HERE, f"{name}_kat.json")) as fh:
        return json.load(fh)
