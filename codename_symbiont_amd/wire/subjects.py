"""NATS subjects of the reference, unchanged for wire compatibility."""
PERCEIVE_URL = "tasks.perceive.url"                     # api_service/src/main.rs:20
RAW_TEXT_DISCOVERED = "data.raw_text.discovered"        # perception_service/src/main.rs:13
TEXT_WITH_EMBEDDINGS = "data.text.with_embeddings"      # preprocessing_service/src/main.rs:16
EMBEDDING_FOR_QUERY = "tasks.embedding.for_query"       # preprocessing_service/src/main.rs:17
SEARCH_SEMANTIC_REQUEST = "tasks.search.semantic.request"  # vector_memory_service/src/main.rs:21
GENERATE_TEXT = "tasks.generation.text"                 # text_generator_service/src/main.rs:10
TEXT_GENERATED = "events.text.generated"                # text_generator_service/src/main.rs:11
PROCESSED_TEXT_TOKENIZED = "data.processed_text.tokenized"  # knowledge_graph_service/src/main.rs:9
QDRANT_COLLECTION_NAME = "symbiont_document_embeddings"  # vector_memory_service/src/main.rs:20
