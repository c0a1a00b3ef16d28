"""Utf8Test.testIsValid (:107-207) restated as vectorised sweeps over the oracle DFA (CPU)."""
import numpy as np


def one_byte(b1, v):
    return np.stack([((b1 << 7) | v)], axis=-1).astype(np.uint8)


def two_byte(b1, b2, v):
    # Utf8Test.twoByte :47-54
    return np.stack([0x80 | (b1 << 5) | ((v >> 6) & 0x1F), (b2 << 6) | (v & 0x3F)], axis=-1).astype(np.uint8)


def three_byte(b1, b2, b3, v):
    # Utf8Test.threeByte :56-65
    return np.stack([0xC0 | (b1 << 4) | ((v >> 12) & 0x0F), (b2 << 6) | ((v >> 6) & 0x3F),
                     (b3 << 6) | (v & 0x3F)], axis=-1).astype(np.uint8)


def four_byte(b1, b2, b3, b4, v):
    # Utf8Test.fourByte :67-78
    return np.stack([0xE0 | (b1 << 3) | ((v >> 18) & 0x07), (b2 << 6) | ((v >> 12) & 0x3F),
                     (b3 << 6) | ((v >> 6) & 0x3F), (b4 << 6) | (v & 0x3F)], axis=-1).astype(np.uint8)


def check(oracle, strings, expected):
    n, w = strings.shape
    got = oracle.utf8_is_valid_batch(strings, np.full(n, w))
    np.testing.assert_array_equal(got, expected)
    # assertIsValidIncomplete :84-105: every proper prefix is invalid
    for ln in range(1, w):
        assert not oracle.utf8_is_valid_batch(strings[:, :ln], np.full(n, ln)).any()


def test_one_byte(oracle):
    v = np.arange(0x80)
    check(oracle, one_byte(0, v), np.ones(0x80, bool))
    check(oracle, one_byte(1, v), np.zeros(0x80, bool))


def test_two_byte(oracle):
    for i in range(4):
        for j in range(4):
            if i == 2 and j == 2:
                v = np.arange(0, 0x80)
                check(oracle, two_byte(i, j, v), np.zeros(v.size, bool))
                v = np.arange(0x80, 0x7FF)
                check(oracle, two_byte(i, j, v), np.ones(v.size, bool))
            else:
                v = np.arange(0, 0x7FF)
                check(oracle, two_byte(i, j, v), np.zeros(v.size, bool))


def test_three_byte(oracle):
    for i in range(4):
        for j in range(4):
            for k in range(4):
                if i == 2 and j == 2 and k == 2:
                    v = np.arange(0, 0x10000)
                    exp = ((v >= 0x800) & (v < 0xD800)) | (v > 0xDFFF)
                    check(oracle, three_byte(i, j, k, v), exp)
                elif i > 1:
                    v = np.arange(0, 0xFFFF)
                    check(oracle, three_byte(i, j, k, v), np.zeros(v.size, bool))


def test_four_byte(oracle):
    v = np.arange(0, 0x200000)
    exp = (v >= 0x10000) & (v <= 0x10FFFF)
    check(oracle, four_byte(2, 2, 2, 2, v), exp)


def test_offset_window(oracle):
    # Utf8Test :193-206 on df df bf df df
    out = bytes([0xDF, 0xDF, 0xBF, 0xDF, 0xDF])
    assert not oracle.utf8_is_valid(out)
    for off in range(5):
        for ln in range(1, 5 - off):
            assert oracle.utf8_is_valid(out[off:off + ln]) == (ln == 2 and off == 1)


def test_dfa_matches_python_strict_decoder_on_random_strings(oracle):
    """Independent cross-check: whole-string verdicts equal CPython's strict UTF-8 decoder."""
    rng = np.random.default_rng(1)
    for w in (1, 2, 3, 4, 5, 8):
        s = rng.integers(0, 256, size=(20000, w), dtype=np.uint8)
        s[s.sum(axis=1) % 3 == 0] |= 0x80  # bias toward high bytes
        got = oracle.utf8_is_valid_batch(s, np.full(len(s), w))
        exp = []
        for row in s:
            try:
                row.tobytes().decode("utf-8", "strict")
                exp.append(True)
            except UnicodeDecodeError:
                exp.append(False)
        np.testing.assert_array_equal(got, np.array(exp))


def test_oracle_validator_context_rule(oracle):
    """FrameUtf8Validator.java:63-95 in any frame order: BINARY leaves an open
    context alone, TEXT continues it, an orphan CONTINUATION is not validated."""
    v = oracle.Validator()
    assert [v.decode(*f) for f in [(1, False, b"\xdf"), (2, True, b"\xff"), (0, True, b"\xdf\xdf")]] == [True, True, False]
    v = oracle.Validator()
    assert [v.decode(*f) for f in [(1, False, b"\xe2\x82"), (1, True, b"\xac")]] == [True, True]
    v = oracle.Validator()
    assert [v.decode(*f) for f in [(0, False, b"\xff"), (0, True, b"\xff"), (1, True, b"ok")]] == [True, True, True]
