"""MI355X-native drop-in for the ska_sdp_func Python package (hot path).

Mirrors the reference package layout (src/ska_sdp_func/ of ska-sdp-func
1.2.2) for the functions on the gridding / degridding hot path; the compiled
library behind it is this repository's HIP build of libska_sdp_func.
"""
