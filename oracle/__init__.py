"""CPU oracle for the HPACK Huffman hot path -- TEST INFRASTRUCTURE ONLY.

Importable only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  See huff_oracle.c for the reference citations.
"""
