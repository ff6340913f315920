"""motion_detection_amd -- MI355X-native flow + egomotion-warp + frame-difference path.

Drop-in for the hot path of shadimsaleh/motion_detection
(OpticalFlowCalculator::calculateOpticalFlow, common/src/optical_flow_calculator.cpp:30-130):
HIP kernels for gfx950 behind the C-ABI in include/mdx.h (libmdx.so), with this package as
the Python host mirroring the reference's interface.
"""
from ._lib import (FIT_EXTERNAL, FIT_FIRST4, FIT_RANSAC, FMT_BGR8, FMT_GRAY8, FMT_RGB8, LIB_PATH, MDX_EDEGENERATE,
                   MDX_OK, SUBSPACE_F32, SUBSPACE_F64, MdxError, MdxParams, build, default_params, lib)
from .context import Context, FlowResult, grid_count, grid_points, host_empty, synth_pair
from .optical_flow_calculator import OpticalFlowCalculator
from .outlier_detector import OutlierDetector

__all__ = ["build", "lib", "Context", "FlowResult", "OpticalFlowCalculator", "OutlierDetector", "MdxError", "MdxParams",
           "default_params", "grid_count", "grid_points", "host_empty", "synth_pair", "LIB_PATH", "FMT_GRAY8", "FMT_RGB8",
           "FMT_BGR8", "FIT_FIRST4", "FIT_EXTERNAL", "FIT_RANSAC", "SUBSPACE_F64", "SUBSPACE_F32", "MDX_OK", "MDX_EDEGENERATE"]
