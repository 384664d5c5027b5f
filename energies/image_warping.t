-- As-rigid-as-possible warping of a 2-D image mesh: every pixel carries a position and
-- a rotation angle; neighbouring pixels inside the mesh keep their rest offset up to
-- that rotation, and handle pixels are pulled to their targets. Declaration indices
-- follow the reference example (examples/image_warping), so its problemparams bind
-- unchanged.
local cols, rows = Dim("W", 0), Dim("H", 1)

local warped    = Unknown("Offset", opt_float2, {cols, rows}, 0)
local theta     = Unknown("Angle", opt_float, {cols, rows}, 1)
local restPos   = Array("UrShape", opt_float2, {cols, rows}, 2)
local handles   = Array("Constraints", opt_float2, {cols, rows}, 3)   -- < 0: no handle
local outside   = Array("Mask", opt_float, {cols, rows}, 4)           -- 0 = pixel of the mesh
local fitW      = Param("w_fitSqrt", float, 5)
local rigidW    = Param("w_regSqrt", float, 6)

UsePreconditioner(true)
Exclude(Not(eq(outside(0, 0), 0)))

local neighbours = Stencil { {1, 0}, {-1, 0}, {0, 1}, {0, -1} }
for ox, oy in neighbours do
    local restEdge = restPos(0, 0) - restPos(ox, oy)
    local residual = (warped(0, 0) - warped(ox, oy)) - Rotate2D(theta(0, 0), restEdge)
    local bothInside = InBounds(ox, oy) * eq(outside(ox, oy), 0) * eq(outside(0, 0), 0)
    Energy(Select(bothInside, rigidW * residual, 0))
end

local isHandle = All(greatereq(handles(0, 0), 0))
Energy(fitW * Select(isHandle, warped(0, 0) - handles(0, 0), 0.0))
