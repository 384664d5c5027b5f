-- Poisson image editing: inside the mask the result takes the gradients of the inserted
-- image; outside it stays fixed. Declaration indices follow the reference example
-- (examples/poisson_image_editing).
local cols, rows = Dim("W", 0), Dim("H", 1)
local result = Unknown("X", opt_float4, {cols, rows}, 0)
local insert = Array("T", opt_float4, {cols, rows}, 1)
local fixed = Array("M", opt_float, {cols, rows}, 2)     -- 0: free pixel
UsePreconditioner(false)
Exclude(Not(eq(fixed(0, 0), 0)))

local function gradient(img, ox, oy) return img(0, 0) - img(ox, oy) end

for ox, oy in Stencil { {1, 0}, {-1, 0}, {0, 1}, {0, -1} } do
    Energy(Select(InBounds(ox, oy), gradient(result, ox, oy) - gradient(insert, ox, oy), 0))
end
