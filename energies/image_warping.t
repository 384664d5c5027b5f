-- As-rigid-as-possible 2-D image warping (same energy as the reference's
-- examples/image_warping/image_warping.t, without its debug printing).
local W, H = Dim("W", 0), Dim("H", 1)

local Offset      = Unknown("Offset", opt_float2, {W, H}, 0)   -- warped position
local Angle       = Unknown("Angle", opt_float, {W, H}, 1)     -- per-pixel rotation
local UrShape     = Array("UrShape", opt_float2, {W, H}, 2)    -- rest position
local Constraints = Array("Constraints", opt_float2, {W, H}, 3) -- handle targets (<0: none)
local Mask        = Array("Mask", opt_float, {W, H}, 4)         -- 0 = part of the mesh
local w_fitSqrt   = Param("w_fitSqrt", float, 5)
local w_regSqrt   = Param("w_regSqrt", float, 6)

UsePreconditioner(true)
Exclude(Not(eq(Mask(0, 0), 0)))

-- rigidity of every 4-neighbour edge inside the mesh
for x, y in Stencil { {1, 0}, {-1, 0}, {0, 1}, {0, -1} } do
    local edge = (Offset(0, 0) - Offset(x, y)) - Rotate2D(Angle(0, 0), UrShape(0, 0) - UrShape(x, y))
    local inside = InBounds(x, y) * eq(Mask(x, y), 0) * eq(Mask(0, 0), 0)
    Energy(Select(inside, w_regSqrt * edge, 0))
end

-- handle constraints
local has = All(greatereq(Constraints(0, 0), 0))
Energy(w_fitSqrt * Select(has, Offset(0, 0) - Constraints(0, 0), 0.0))
