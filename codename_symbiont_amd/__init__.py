"""codename_symbiont_amd -- an MI355X-native semantic-ingest and vector-search system.

Capabilities of makkenzo/codename-symbiont (same HTTP/SSE API, NATS subjects, JSON wire shapes and
Neo4j graph format), re-designed for AMD Instinct MI355X (gfx950 / CDNA4):

* ``models``   sentence-transformer encoder families (MiniLM-L6, bge-base, e5-large, mpnet-multi)
               executed by hand-written HIP kernels (MFMA GEMMs, varlen attention, fused LN/pool)
* ``ops``      typed front-ends of the HIP kernels + fp32 PyTorch oracles
* ``index``    in-HBM brute-force cosine top-k index (fused MFMA scan + top-k), payloads, WAL
* ``parallel`` one-process-per-GPU data parallel encoding and index sharding over RCCL/xGMI
* ``wire``     the 15 wire contracts of the reference (byte-compatible JSON)
* ``bus``      NATS protocol client + in-repo broker
* ``text``     WordPiece tokenizer, sentence splitter, HTML text extractor, Markov generator
* ``kg``       Bolt/PackStream client for the Neo4j knowledge graph
* ``services`` api / perception / preprocessing / vector_memory / text_generator / knowledge_graph
"""
__version__ = "0.1.0"
