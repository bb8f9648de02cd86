"""Oracle restatement of the validator's TP matching (TEST INFRASTRUCTURE ONLY).

box_iou follows U/utils/metrics.py:52-71 and match_predictions the non-scipy branch of
U/engine/validator.py:222-262, as called by DetectionValidator._process_batch
(U/models/yolo/detect/val.py:209-227).  The checker for ydbl_match_predictions; only tests/
import it.
"""

from __future__ import annotations

import numpy as np
import torch

IOUV = torch.linspace(0.5, 0.95, 10)  # U/models/yolo/detect/val.py:36


def box_iou(box1: torch.Tensor, box2: torch.Tensor, eps: float = 1e-7) -> torch.Tensor:
    """U/utils/metrics.py:52-71: pairwise IoU of xyxy boxes, [N, M]."""
    (a1, a2), (b1, b2) = box1.float().unsqueeze(1).chunk(2, 2), box2.float().unsqueeze(0).chunk(2, 2)
    inter = (torch.min(a2, b2) - torch.max(a1, b1)).clamp_(0).prod(2)
    return inter / ((a2 - a1).prod(2) + (b2 - b1).prod(2) - inter + eps)


def match_predictions(pred_classes: torch.Tensor, true_classes: torch.Tensor, iou: torch.Tensor,
                      iouv: torch.Tensor = IOUV) -> torch.Tensor:
    """U/engine/validator.py:222-262 (non-scipy branch). iou: [labels, detections]."""
    correct = np.zeros((pred_classes.shape[0], iouv.shape[0])).astype(bool)
    correct_class = true_classes[:, None] == pred_classes
    iou = (iou * correct_class).cpu().numpy()
    for i, threshold in enumerate(iouv.cpu().tolist()):
        matches = np.nonzero(iou >= threshold)
        matches = np.array(matches).T
        if matches.shape[0]:
            if matches.shape[0] > 1:
                matches = matches[iou[matches[:, 0], matches[:, 1]].argsort()[::-1]]
                matches = matches[np.unique(matches[:, 1], return_index=True)[1]]
                matches = matches[np.unique(matches[:, 0], return_index=True)[1]]
            correct[matches[:, 1].astype(int), i] = True
    return torch.tensor(correct, dtype=torch.bool, device=pred_classes.device)
