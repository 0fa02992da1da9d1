"""RQ presets of the reference (config.py:42-58; config_optimized.py:62-78 has TEST = [32,128,128]).
Only the semantic-ID presets are mirrored: the T5 / Word2Vec / DDP settings are out of scope."""
from .hierarchical_rq_kmeans import HierarchicalRQKMeansConfig

H_RQ_KMEANS_PROD = HierarchicalRQKMeansConfig(layer_clusters=[128, 1280, 1280], need_clusters=[128, 128, 256],
                                              embedding_dim=512, group_dims=[512],
                                              hierarchical_weights=[[1.0], [1.0], [1.0]], iter_limit=100)
H_RQ_KMEANS_TEST = HierarchicalRQKMeansConfig(layer_clusters=[32, 64, 64], need_clusters=[32, 32, 32],
                                              embedding_dim=512, group_dims=[512],
                                              hierarchical_weights=[[1.0], [1.0], [1.0]], iter_limit=50)
H_RQ_KMEANS_TEST_OPTIMIZED = HierarchicalRQKMeansConfig(layer_clusters=[32, 128, 128], need_clusters=[32, 32, 32],
                                                        embedding_dim=512, group_dims=[512],
                                                        hierarchical_weights=[[1.0], [1.0], [1.0]], iter_limit=50)
# BASELINE.json configs[4]: [256,256,512] with layer_clusters in the PROD ratios
H_RQ_KMEANS_XL = HierarchicalRQKMeansConfig(layer_clusters=[256, 2560, 2560], need_clusters=[256, 256, 512],
                                            embedding_dim=512, group_dims=[512],
                                            hierarchical_weights=[[1.0], [1.0], [1.0]], iter_limit=100)
