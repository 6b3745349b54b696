"""Known-answer tests for the oracle, derived by hand from the reference source.

Each expected value is worked out from the cited reference lines, independently of the
oracle code; together with tests/pyref.py they are what pins the oracle (the reference
itself cannot be built here and ships no fixtures — see oracle/oracle.cpp header).
"""
import numpy as np
import pytest

import oracle
import pyref


def test_kmer_iterator_basic_positions():
    # KmerIterator.cpp:65-76 — A0 C1 G2 T3, first base in the high bits, canonical =
    # min(fwd, rc), position_in_sequence is end-exclusive after next_kmer().
    # "ACGT", k=2: AC fwd 0b0001=1 rc(GT)=0b1011=11 -> 1 @2; CG 6/6 -> 6 @3; GT 11 rc(AC)=1 -> 1 @4
    codes, pos = oracle.kmer_windows(b"ACGT", 2)
    assert codes.tolist() == [1, 6, 1]
    assert pos.tolist() == [2, 3, 4]


def test_kmer_iterator_short_read_and_exact_k():
    # KmerIterator.cpp:33-34: a read shorter than k yields nothing; len == k yields one window.
    assert len(oracle.kmer_windows(b"ACG", 4)[0]) == 0
    codes, pos = oracle.kmer_windows(b"ACGT", 4)
    assert pos.tolist() == [4]
    assert codes.tolist() == [min(0b00011011, 0b00011011)]  # ACGT is its own reverse complement


def test_kmer_iterator_non_acgt_quirk():
    # BASE_TO_NUM / COMPLEMENT are unordered_map::operator[]: 'N' -> 0 on BOTH strands
    # (KmerIterator.cpp:7-19,56,62).  "TNT", k=2: prime T: fwd=3 rc=0; N: fwd=12, rc=0 -> 0 @2;
    # T: fwd=(12<<2|3)&15=3, rc=0 -> 0 @3.  (A reverse-complement-consistent code of "TA"
    # would be 12.)
    codes, pos = oracle.kmer_windows(b"TNT", 2)
    assert codes.tolist() == [0, 0]
    assert pos.tolist() == [2, 3]
    # lower-case is not a base for KmerIterator either: "aC", k=2 -> fwd 0b0001=1, rc = C's
    # complement G(1)<<2 | 0 = 4 -> min 1
    codes, _ = oracle.kmer_windows(b"aC", 2)
    assert codes.tolist() == [1]


def test_kmer_iterator_k32_and_k_too_big():
    seq = b"T" * 32
    codes, _ = oracle.kmer_windows(seq, 32)
    assert codes.tolist() == [0]          # fwd = all ones, rc = poly-A = 0
    with pytest.raises(ValueError):
        oracle.kmer_windows(b"A" * 40, 33)  # KmerIterator.cpp:24-26 throws


def test_jellyfish_count_semantics():
    # run_jellyfish.sh: canonical (-C), exact counts, singletons dropped (--bc), windows
    # with non-ACGT skipped, lower-case counted as bases.  Hand count, k=2:
    #   "ACGT" -> AC:1 CG:6 GT->1 : {1:2, 6:1}, three runs ("ACGT","ACGT","acgt") -> {1:6, 6:3}
    keys, counts = oracle.count_stream(b"ACGTNACGT\nacgt", 2, 2)
    assert keys.tolist() == [1, 6]
    assert counts.tolist() == [6, 3]
    keys, counts = oracle.count_stream(b"ACGA", 2, 2)   # AC:1 CG:6 GA->TC=13 rc... each once
    assert keys.tolist() == []
    keys, counts = oracle.count_stream(b"ACGA", 2, 1)
    # GA fwd 0b1000=8, rc(GA)=TC=0b1101=13 -> 8
    assert dict(zip(keys.tolist(), counts.tolist())) == {1: 1, 6: 1, 8: 1}


def test_merge_fills_missing_with_zero():
    # get_next_kmer (JellyfishOccurrenceReader.cpp:63-86): counts[f] = 0 when file f lacks it.
    keys, counts = oracle.merge([(np.array([1, 5], np.uint64), np.array([2, 3], np.uint32)),
                                 (np.array([5, 9], np.uint64), np.array([4, 7], np.uint32))])
    assert keys.tolist() == [1, 5, 9]
    assert counts.tolist() == [[2, 0], [3, 4], [0, 7]]


def test_specificity_bins_by_hand():
    # JellyfishOccurrenceReader.cpp:88-108 with thresholds {70,85,90,95,99,100,100.01}:
    #   [5,0] 100%   -> upper_bound(100)  = 100.01 (idx 6)
    #   [3,1] 75%    -> 85 (idx 1);  [7,3] exactly 70.0 -> 85 (upper_bound is strict)
    #   [1,1] 50%    -> 70 (idx 0);  [99,1] 99% -> 100 (idx 5); [2,1] 66.7% -> 70
    rows = np.array([[5, 0], [3, 1], [7, 3], [1, 1], [99, 1], [2, 1]], np.uint32)
    h = oracle.specificity(rows, oracle.THRESHOLDS).tolist()
    assert h == [[0, 2, 1], [0, 3, 1], [1, 4, 1], [1, 10, 1], [5, 100, 1], [6, 5, 1]]


def test_select_and_discriminative():
    # export_kmers (:110-135): lower <= total <= upper; discriminative = one nonzero file.
    keys = np.array([1, 2, 3, 4], np.uint64)
    counts = np.array([[10, 0], [5, 6], [30, 0], [0, 25]], np.uint32)
    sel, d = oracle.select(keys, counts, 10, 25)
    assert sel.tolist() == [1, 2, 4]
    assert d == 2


def test_sdk_text_load():
    # load_text_file_kmers (read_clustering.cpp:18-33): k = last line length; canonical code.
    keys, k = oracle.load_sdk_text(b"ACGT\nTTTT\n")
    assert k == 4
    assert sorted(keys.tolist()) == [0, 0b00011011]   # TTTT canonicalises to AAAA = 0


def test_pyref_agrees_with_hand_values():
    assert [c for c, _ in pyref.kmer_iterator("TNT", 2)] == [0, 0]
    assert pyref.jf_count("ACGTNACGT\nacgt", 2) == [(1, 6), (6, 3)]
