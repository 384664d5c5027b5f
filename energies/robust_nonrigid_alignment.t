-- Robust non-rigid alignment (same energy as the reference's
-- examples/robust_nonrigid_alignment; same declaration indices): ARAP regularisation of
-- a template deformed towards point-to-plane correspondences, each correspondence with
-- a per-vertex confidence that is itself optimised (and pulled towards 1).
local N = Dim("N", 0)
local NUMEDGES = Dim("NUMEDGES", 1)

local w_fit = Param("w_fitSqrt", float, 0)
local w_reg = Param("w_regSqrt", float, 1)
local w_conf = 0.1
local Offset  = Unknown("Offset", opt_float3, {N}, 2)
local Angle   = Unknown("Angle", opt_float3, {N}, 3)
local Weight  = Unknown("RobustWeights", opt_float, {N}, 4)
local UrShape = Array("UrShape", opt_float3, {N}, 5)
local Target  = Array("Constraints", opt_float3, {N}, 6)          -- < -999999.9: none
local Normal  = Array("ConstraintNormals", opt_float3, {N}, 7)
local G = Graph("G", {NUMEDGES}, "v0", {N}, 9, "v1", {N}, 10)
UsePreconditioner(true)

local w = Weight(0)
local has = greatereq(Target(0), -999999.9)
Energy(w_fit * Select(has, w * Normal(0):dot(Offset(0) - Target(0)), 0.0))
Energy(w_conf * Select(has, 1 - w * w, 0.0))

local rigid = (Offset(G.v0) - Offset(G.v1)) - Rotate3D(Angle(G.v0), UrShape(G.v0) - UrShape(G.v1))
Energy(w_reg * rigid)
