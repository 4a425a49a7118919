// wf_vol.hip — one variant group of the wavefront pipeline (ring 8, rare-primitive (volume / circle / reference-order) kernels),
// instantiated in its own translation unit so the groups compile in parallel
// (wavefront.hip, RTG_WF_GROUP).
#define RTG_WF_GROUP 1
#include "wavefront.hip"
