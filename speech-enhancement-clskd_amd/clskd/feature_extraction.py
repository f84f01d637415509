"""feature_extraction.py drop-in (local-DCCRN taps, feature_extraction.py:3-50).

``DCCRN(model).extract_feature_maps(x)`` returns the same dict as the reference:
``{"encoder": [6 NCHW], "decoder": [6 NCHW, before [...,1:]], "clstm": [[real, imag] (T,B,D)]}``.
The reference registers forward hooks; ``clskd.DCCRN`` runs as one HIP executor, so the taps are
delivered through a tap sink instead (same lifetime semantics: ``remove_hook`` detaches it).
"""
from .model import DCCRN as _DCCRNModel


class DCCRN:
    def __init__(self, model):
        if not isinstance(model, _DCCRNModel):
            raise TypeError("feature_extraction.DCCRN expects a clskd.DCCRN model")
        self.model = model
        self.feature_maps = {"encoder": [], "decoder": [], "clstm": []}
        self._sink = self._collect
        model._tap_sinks.append(self._sink)

    def _collect(self, res):
        self.feature_maps["encoder"].extend(res["enc_nchw"])
        self.feature_maps["decoder"].extend(res["dec_nchw"])
        self.feature_maps["clstm"].append(list(_DCCRNModel.clstm_from_dec_in(res["dec_in"])))

    def remove_hook(self):
        if self._sink in self.model._tap_sinks:
            self.model._tap_sinks.remove(self._sink)

    def extract_feature_maps(self, input):
        self.model(input)
        return self.feature_maps
