-- Intrinsic image decomposition in log space: the image i is explained as
-- reflectance r (RGB) plus shading s (grey), i = r + s. Reflectance differences get an
-- iteratively reweighted L_p prior (the weights come from r_const, a view of r declared on
-- the same parameter slot, through a ComputedArray refreshed after every update), shading
-- differences an L_2 prior. Same energy as the reference's
-- examples/intrinsic_image_decomposition; runs on the generated kernels.
local W, H = Dim("W", 0), Dim("H", 1)

local w_fit     = Param("w_fitSqrt", float, 0)
local w_albedo  = Param("w_regSqrtAlbedo", float, 1)
local w_shading = Param("w_regSqrtShading", float, 2)
local p_norm    = Param("pNorm", opt_float, 3)
local r         = Unknown("r", opt_float3, {W, H}, 4)
local r_const   = Array("r_const", opt_float3, {W, H}, 4)
local i         = Array("i", opt_float3, {W, H}, 5)
local s         = Unknown("s", opt_float, {W, H}, 6)

local neighbours = { {1, 0}, {-1, 0}, {0, 1}, {0, -1} }

for _, d in ipairs(neighbours) do
    local dx, dy = d[1], d[2]
    local weighted = L_p(r(0, 0) - r(dx, dy), r_const(0, 0) - r_const(dx, dy), p_norm, {W, H})
    Energy(w_albedo * Select(InBounds(0, 0), Select(InBounds(dx, dy), weighted, 0), 0))
end

for _, d in ipairs(neighbours) do
    local dx, dy = d[1], d[2]
    Energy(w_shading * Select(InBounds(0, 0), Select(InBounds(dx, dy), s(0, 0) - s(dx, dy), 0), 0))
end

Energy(w_fit * (r(0, 0) + s(0, 0) - i(0, 0)))
