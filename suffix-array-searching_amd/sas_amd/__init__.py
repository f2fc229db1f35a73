"""sas_amd -- MI355X-native batched suffix-array / static-search-tree lookup.

Host-side mirror of the reference's query API (RagnarGrootKoerkamp/suffix-array-searching)
over the C ABI of libsas_amd.so (include/sas.h, include/sst.h).
"""
from ._lib import SasError, lib, build_library, declared_symbols, LIB_PATH, source_hash  # noqa: F401
from .sa import (SaNaive, Counter, binary_search, binary_search_batch,  # noqa: F401
                 random_string, random_queries, read_fasta_file, kmer_keys)
from .multi import SaMulti  # noqa: F401
from .sst import (SortedVec, Eytzinger, STree16, STree15, PartitionedSTree16M, DirectMap, MAX,  # noqa: F401
                  PartitionedSTree16, PartitionedSTree16C, PartitionedSTree16L, PartitionedSTree16O)
