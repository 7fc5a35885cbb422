"""Drop-in mirrors of the reference's ``layers`` package (same class names,
constructor arguments and parameter names), executing on librgbac_hip.so."""
