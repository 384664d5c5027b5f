-- Dense optical flow: X(i,j) moves pixel (i,j) of I onto the sampled target I_hat,
-- with a 4-neighbour smoothness prior (same energy as the reference's
-- examples/optical_flow/optical_flow.t).
local W, H = Dim("W", 0), Dim("H", 1)
local w_fitSqrt = Param("w_fit", float, 0)
local w_regSqrt = Param("w_reg", float, 1)
local X = Unknown("X", opt_float2, {W, H}, 2)          -- flow vectors
local I = Array("I", opt_float, {W, H}, 3)             -- source image
local target = Array("I_hat", opt_float, {W, H}, 4)    -- target image
local target_dx = Array("I_hat_dx", opt_float, {W, H}, 5)
local target_dy = Array("I_hat_dy", opt_float, {W, H}, 6)
local I_hat = SampledImage(target, target_dx, target_dy)   -- bilinear, with its derivatives

local i, j = Index(0), Index(1)
UsePreconditioner(false)

Energy(w_fitSqrt * (I(0, 0) - I_hat(i + X(0, 0, 0), j + X(0, 0, 1))))

for dx, dy in Stencil { {1, 0}, {-1, 0}, {0, 1}, {0, -1} } do
    local smooth = w_regSqrt * (X(0, 0) - X(dx, dy))
    Energy(Select(InBounds(dx, dy), smooth, 0))
end
