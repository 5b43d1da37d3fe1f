"""Drop-in for speechbrain.nnet.transducer.transducer_joint.Transducer_joint
(transducer_joint.py:14-95).

joint="sum" (the LibriSpeech transducer recipe, train.yaml:179-181): the
broadcast add TN (B, T, 1, J) + PN (B, 1, U+1, J) and the nonlinearity run as
one HIP kernel (sbk_joint_fwd) writing (B, T, U+1, J) directly — in bf16
under autocast, so the largest activation of the step is half-size — with the
backward reductions over U (dTN) and T (dPN) in csrc/backward.hip.
joint="concat" expands and concatenates (layout only) and applies
joint_network, as the reference does (:75-93).
"""
import torch
import torch.nn as nn

from ... import _autograd as A
from ... import _enc

_ACT = {nn.Identity: 0, nn.LeakyReLU: 3, nn.Tanh: 5, nn.ReLU: 6}


class Transducer_joint(nn.Module):
    def __init__(self, joint_network=None, joint="sum", nonlinearity=torch.nn.LeakyReLU):
        super().__init__()
        self.joint_network = joint_network
        self.joint = joint
        self.nonlinearity = nonlinearity()

    def init_params(self, first_input):
        self.joint_network(first_input)

    def _act(self):
        code = _ACT.get(type(self.nonlinearity))
        if code is None:
            raise NotImplementedError(f"joint nonlinearity {type(self.nonlinearity).__name__} has no HIP kernel")
        slope = getattr(self.nonlinearity, "negative_slope", 0.0) if code == 3 else 0.0
        return code, slope

    def forward(self, input_TN, input_PN):
        if len(input_TN.shape) != len(input_PN.shape):
            raise ValueError("Arg 1 and 2 must be have same size")
        if self.joint == "sum" and input_TN.dim() == 4 and input_TN.shape[2] == 1 and input_PN.shape[1] == 1:
            code, slope = self._act()
            out_dtype = _enc.compute_dtype()
            tn = input_TN[:, :, 0, :]
            pn = input_PN[:, 0, :, :]
            return A.JointFn.apply(A.to_dtype(tn.float(), torch.float32), A.to_dtype(pn.float(), torch.float32),
                                   code, slope, out_dtype)
        if self.joint == "sum":
            joint = input_TN + input_PN
        elif self.joint == "concat":
            if input_TN.dim() == 4:
                sz = [max(i, j) for i, j in zip(input_TN.size()[:-1], input_PN.size()[:-1])]
                xs = input_TN.expand(torch.Size(sz + [input_TN.shape[-1]]))
                ys = input_PN.expand(torch.Size(sz + [input_PN.shape[-1]]))
                joint = torch.cat((xs, ys), dim=3)
            elif input_TN.dim() == 1:
                joint = torch.cat((input_TN, input_PN), dim=0)
            else:
                raise ValueError("Tensors 1 and 2 must have dim=1 or dim=4")
            if self.joint_network is not None:
                joint = self.joint_network(joint)
        else:
            raise ValueError(f"unknown joint {self.joint}")
        return self.nonlinearity(joint)
