"""mast3r_slam.monst3r_utils (monst3r_utils.py:36-782) on the MI355X pair model."""
from monst3r_slam_amd.monst3r_utils import (Frame, ModelHandle, apply_dynamic_mask_to_pointmaps,  # noqa: F401
                                            create_frame, dynamic_mask_from_flow, ego_flow,
                                            get_dynamic_mask, load_mast3r, load_monst3r,
                                            monst3r_asymmetric_inference,
                                            monst3r_asymmetric_inference_with_dynamic_mask,
                                            monst3r_decode_symmetric_batch,
                                            monst3r_match_asymmetric_with_dynamic_mask,
                                            monst3r_inference_mono, monst3r_match_asymmetric,
                                            monst3r_symmetric_inference, resize_img,
                                            sim3_relative_matrix)
from monst3r_slam_amd import monst3r_utils as _U
from monst3r_slam_amd.retrieval import load_retriever  # noqa: F401


def monst3r_match_symmetric(mast3r=None, monst3r=None, feat_i=None, pos_i=None, feat_j=None,
                            pos_j=None, shape_i=None, shape_j=None):
    """:214-252.  global_opt2.py:54-59 calls it by keyword without `mast3r` (the
    reference's missing-argument bug): both decoders live in the one MI355X
    pair model, reached from either handle, so the call works either way."""
    return _U.monst3r_match_symmetric(mast3r, monst3r, feat_i, pos_i, feat_j, pos_j, shape_i,
                                      shape_j)

# SAM2 mask refinement (monst3r_utils.py:20-34): its code and checkpoint are absent from the
# reference checkout — the constants keep tracker2.py importable and its own
# checks (os.path.exists on the checkpoint) disable the refinement.
SAM2_CHECKPOINT_DEFAULT = "checkpoints/sam2.1_hiera_large.pt"
SAM2_MODEL_CONFIG_NAME_FOR_HYDRA = "configs/sam2.1/sam2.1_hiera_l.yaml"
SAM2_MODEL_CONFIG_ABSOLUTE_PATH = "thirdparty/sam2/sam2/configs/sam2.1/sam2.1_hiera_l.yaml"


def build_sam2_video_predictor(*args, **kwargs):
    raise NotImplementedError("SAM2 is not part of the MI355X build (absent reference code)")
