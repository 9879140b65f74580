"""Model zoo: reference Models A (MTL_Net), B (Single_Task_Net) and C (Multi_Classifier)."""
from .layers import ResBlock, att_generator, conv3x3, encoder_block
from .mtl import MTL_Net, MTLNet, Single_Task_Net, TASK_CLASSES
from .multi_classifier import (BasicConv2d, InceptionA, InceptionAux, InceptionB, InceptionC, InceptionD,
                               InceptionE, Multi_Classifier, decode_joint, encode_joint)

MODEL_TYPES = ("MTL", "single_distance", "single_event", "multi_classifier")


def build_model(model_type: str, in_channels: int = 1, head: str = "group_mean"):
    """Model factory with the reference's ``--model`` names (reference utils.py:85-98).  ``head="fc"``
    (Models A / B only) is the backbone-vs-head ablation of docs/ACCURACY.md, not a reference model."""
    if model_type == "multi_classifier":
        if head != "group_mean":
            raise ValueError("--head applies to the MTL / single-task models only")
        return Multi_Classifier(in_channels=in_channels)
    if model_type == "MTL":
        return MTL_Net(in_channels=in_channels, head=head)
    if model_type == "single_distance":
        return Single_Task_Net("distance", in_channels=in_channels, head=head)
    if model_type == "single_event":
        return Single_Task_Net("event", in_channels=in_channels, head=head)
    raise ValueError(f"unknown model type {model_type!r}; expected one of {MODEL_TYPES}")


def model_tasks(model_type: str):
    """The (task, n_classes) list a model predicts; multi_classifier predicts the 32-way joint label."""
    return {"MTL": [("distance", 16), ("event", 2)], "single_distance": [("distance", 16)],
            "single_event": [("event", 2)], "multi_classifier": [("joint", 32)]}[model_type]
