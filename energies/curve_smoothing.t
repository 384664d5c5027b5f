-- Polyline fairing in 3-D: points stay near their samples while consecutive
-- segments keep a rest length and the discrete curvature is damped (nonlinear:
-- the length term goes through a square root). Runs on generated kernels.
local N = Dim("N", 0)

local P        = Unknown("P", opt_float3, {N}, 0)     -- fitted points
local S        = Array("S", opt_float3, {N}, 1)       -- noisy samples
local w_fit    = Param("w_fit", float, 2)
local w_len    = Param("w_len", float, 3)
local w_bend   = Param("w_bend", float, 4)
local rest     = Param("rest", float, 5)

local function segment(a, b) return P(b) - P(a) end

Energy(w_fit * (P(0) - S(0)))
local seg = segment(0, 1)
Energy(Select(InBounds(1), w_len * (sqrt(Dot3(seg, seg)) - rest), 0))
Energy(Select(InBounds(-1) * InBounds(1), w_bend * (P(-1) - 2 * P(0) + P(1)), 0))
