"""End-to-end algorithm tests on the MI355X: the CPU suites' doc / golden tests re-run with the default
environment on cuda:0 (MLEnvironment picks the rank's GPU when one is present), so the driver's ``-m gpu`` run
covers every algorithm family through its device path (HIP kernels where they exist, torch on the device
otherwise), not only the kernel unit tests."""
import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [
    ("test_kmeans", "test_kmeans_pipeline_distances"),
    ("test_kmeans", "test_kmeans_model_mapper_detail"),
    ("test_kmeans", "test_kmeans_blobs_converges_and_recovers_centers"),
    ("test_linear", "test_linear_regression_doc_example"),
    ("test_linear", "test_ridge_regression_doc_example"),
    ("test_linear", "test_softmax_doc_example"),
    ("test_linear", "test_lr_detail_and_model_rows"),
    ("test_linear", "test_aft_doc_example_bitwise"),
    ("test_tree", "test_gbdt_classifier_doc_bit_exact"),
    ("test_tree", "test_gbdt_regressor_and_stream_doc"),
    ("test_tree", "test_random_forest_synthetic"),
    ("test_tree", "test_gbdt_synthetic_accuracy_and_regression"),
    ("test_als", "test_als_topk_stream_and_pipeline"),
    ("test_als", "test_als_recovers_low_rank_matrix"),
    ("test_glm_isotonic", "test_glm_gamma_log_matches_doc"),
    ("test_glm_isotonic", "test_glm_gaussian_identity_is_ols"),
    ("test_glm_isotonic", "test_isotonic_doc_model_and_predictions"),
    ("test_fm", "test_fm_regressor_learns_interaction"),
    ("test_fm", "test_fm_classifier_detail_and_model_format"),
    ("test_nlp", "test_word2vec_doc_and_semantics"),
    ("test_nlp", "test_doc_count_vectorizer_doc_model"),
    ("test_gmm_bisecting", "test_gmm_doc_example"),
    ("test_gmm_bisecting", "test_bisecting_kmeans_doc_example"),
    ("test_mlp", "test_mlpc_iris_accuracy"),
    ("test_pca_chisq", "test_pca_doc_example_batch_stream_pipeline"),
    ("test_evaluation", "test_eval_binary_doc"),
    ("test_evaluation", "test_eval_cluster_doc"),
    ("test_feature", "test_feature_hasher_doc_bitexact"),
    ("test_feature", "test_one_hot_doc"),
    ("test_feature", "test_quantile_discretizer_and_summarizer"),
    ("test_mining", "test_sos_doc"),
    ("test_mining", "test_lsh_doc_and_murmur"),
    ("test_tuning_ovr", "test_one_vs_rest_lr"),
    ("test_ftrl", "test_ftrl_doc_example"),
]


@pytest.mark.parametrize("mod,fn", CASES)
def test_algorithm_on_gpu(mod, fn):
    from alink_amd.common.mlenv import MLEnvironmentFactory
    from alink_amd.ops import _lib
    assert torch.cuda.is_available() and _lib.available()
    assert MLEnvironmentFactory.getDefault().device.type == "cuda"
    getattr(importlib.import_module(mod), fn)()
