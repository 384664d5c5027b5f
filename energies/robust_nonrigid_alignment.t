-- Non-rigid alignment of a template to scan correspondences (point-to-plane), with an
-- optimised per-vertex confidence that is pulled towards 1, regularised as-rigid-as-
-- possible over the template's edges. Declaration indices follow the reference example
-- (examples/robust_nonrigid_alignment).
local nv, ne = Dim("N", 0), Dim("NUMEDGES", 1)

local corrW = Param("w_fitSqrt", float, 0)
local arapW = Param("w_regSqrt", float, 1)
local confW = 0.1
local disp   = Unknown("Offset", opt_float3, {nv}, 2)
local rot    = Unknown("Angle", opt_float3, {nv}, 3)
local conf   = Unknown("RobustWeights", opt_float, {nv}, 4)
local base   = Array("UrShape", opt_float3, {nv}, 5)
local corr   = Array("Constraints", opt_float3, {nv}, 6)
local normal = Array("ConstraintNormals", opt_float3, {nv}, 7)
local E = Graph("G", {ne}, "v0", {nv}, 9, "v1", {nv}, 10)
UsePreconditioner(true)

local c = conf(0)
local matched = greatereq(corr(0), -999999.9)
local planeDist = c * normal(0):dot(disp(0) - corr(0))
Energy(corrW * Select(matched, planeDist, 0.0))
Energy(confW * Select(matched, 1 - c * c, 0.0))

local stretch = (disp(E.v0) - disp(E.v1)) - Rotate3D(rot(E.v0), base(E.v0) - base(E.v1))
Energy(arapW * stretch)
